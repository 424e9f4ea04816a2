#!/bin/bash
# bench (default) + sort debug traces of the main and long-repeat workloads + kernel trace of long-repeat
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
echo "gpu tests $(date)"
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bwt or levels or golden or long_repeat or periodic" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "bench $(date)"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "debug main $(date)"
BZG_DEBUG=1 BZG_ONE_STREAM=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-h2h --no-extra > $O/debug.json 2> $O/debug.err || { echo "debug failed"; exit 1; }
echo "debug repeat $(date)"
BZG_DEBUG=1 BZG_ONE_STREAM=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-h2h --no-extra --repeat-frac 0.25 > $O/debug_rep.json 2> $O/debug_rep.err || { echo "debug rep failed"; exit 1; }
echo "trace $(date)"
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof.log 2>&1 || { echo "trace failed"; exit 1; }
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_rep -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra --repeat-frac 0.25 > $O/prof_rep.log 2>&1 || { echo "trace rep failed"; exit 1; }
echo "done $(date)"
