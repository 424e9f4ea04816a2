#!/bin/bash
# Round-6 (development tool): timing of text / long repeats / PRNG and the small-call probe.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
BZG_CHECK=1 timeout -k 10 300 python tools/prof_config.py text 1 > $O/check_text.log 2>&1 || { echo "check failed"; tail -20 $O/check_text.log; exit 1; }
echo "check text: $(grep -c 'bzg check' $O/check_text.log) bad"
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b_$r.json 2> $O/b_$r.err || { echo "bench failed"; tail $O/b_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$r.json').read().strip().splitlines()[-1]); print('1e9', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  timeout -k 10 300 python tools/small_probe.py > $O/s_$r.log 2>&1 || { echo "probe failed"; tail $O/s_$r.log; exit 1; }
  tail -1 $O/s_$r.log
done
for k in repeat random; do
  timeout -k 10 300 python tools/prof_config.py $k 2 > $O/t_$k.log 2>&1 || { echo "$k failed"; tail -20 $O/t_$k.log; exit 1; }
  grep -E "^$k " $O/t_$k.log
done
echo "done $(date)"
