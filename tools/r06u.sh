#!/bin/bash
# Round-6 (development tool): same-box A/B of an env knob on the text bench and the small probe.
# usage: tools/r06u.sh <tag> VAR valA valB
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O; V=$2
for r in 1 2 3; do
  for val in $3 $4; do
    export $V=$val
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b_${val}_$r.json 2> $O/b_${val}_$r.err || { echo "bench failed"; tail $O/b_${val}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${val}_$r.json').read().strip().splitlines()[-1]); print('$V=$val', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  done
done
for val in $3 $4; do
  export $V=$val
  timeout -k 10 300 python tools/small_probe.py > $O/s_$val.log 2>&1 || { echo "probe failed"; tail $O/s_$val.log; exit 1; }
  echo "$V=$val $(tail -1 $O/s_$val.log)"
  timeout -k 10 300 python tools/prof_config.py repeat 2 > $O/t_$val.log 2>&1 || { echo "repeat failed"; exit 1; }
  echo "$V=$val $(grep -E '^repeat ' $O/t_$val.log)"
done
