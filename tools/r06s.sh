#!/bin/bash
# Round-6 (development tool): launch-count changes (fused S1/S2 helper kernels, single-pass
# scan) -- BZG_CHECK runs, GPU tests, text bench, small-call probe and the 100 MB call's trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for k in text repeat random; do
  BZG_CHECK=1 timeout -k 10 300 python tools/prof_config.py $k 1 > $O/check_$k.log 2>&1 || { echo "check $k failed"; tail -20 $O/check_$k.log; exit 1; }
  echo "check $k: $(grep -c 'bzg check' $O/check_$k.log) bad; $(grep -E "^$k " $O/check_$k.log)"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
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
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/gap_probe.py 100000000 > $O/probe.log 2>&1 || { echo "trace failed"; tail -20 $O/probe.log; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python tools/gap_probe.py --report $f > $O/gaps.txt && head -3 $O/gaps.txt
echo "done $(date)"
