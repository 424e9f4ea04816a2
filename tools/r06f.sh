#!/bin/bash
# Round-6 check run (development tool): the S1 next-pass sizes under BZG_CHECK, GPU tests,
# bench text line, small-call probe.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
BZG_CHECK=1 timeout -k 10 300 python tools/prof_config.py text 1 > $O/check.log 2>&1 || { echo "check run failed"; tail -20 $O/check.log; exit 1; }
echo "check lines: $(grep -c 'bzg check' $O/check.log)"; grep 'bzg check' $O/check.log | head -5
BZG_CHECK=1 timeout -k 10 300 python tools/prof_config.py repeat 1 > $O/check_r.log 2>&1 || { echo "check run failed"; tail -20 $O/check_r.log; exit 1; }
echo "check lines (repeat): $(grep -c 'bzg check' $O/check_r.log)"; grep 'bzg check' $O/check_r.log | head -5
if [ "$2" != notests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b_$r.json 2> $O/b_$r.err || { echo "bench failed"; tail $O/b_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$r.json').read().strip().splitlines()[-1]); print('1e9', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  timeout -k 10 300 python tools/small_probe.py > $O/s_$r.log 2>&1 || { echo "probe failed"; tail $O/s_$r.log; exit 1; }
  tail -1 $O/s_$r.log
done
echo "done $(date)"
