#!/bin/bash
# quick: parity tests subset + debug traces (main, repeat) + kernel trace (main)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-bwt or long_repeat or periodic or levels or golden or edge or deep}" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rf in 0 0.25; do
  BZG_DEBUG=1 BZG_ONE_STREAM=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-h2h --no-extra --repeat-frac $rf > $O/debug_$rf.json 2> $O/debug_$rf.err || exit 1
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-extra --repeat-frac $rf > $O/b_$rf.json 2> $O/b_$rf.err || exit 1
  python3 -c "import json;d=json.load(open('$O/b_$rf.json'));print('rf $rf', d['value'],d['stages_ms'])"
done
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof.log 2>&1 || { echo "trace failed"; exit 1; }
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_rep -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra --repeat-frac 0.25 > $O/prof_rep.log 2>&1 || { echo "trace failed"; exit 1; }
echo "done $(date)"
