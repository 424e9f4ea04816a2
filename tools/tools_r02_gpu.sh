#!/bin/bash
# one GPU call: gpu tests, default bench (secondary lines included), a BZG_DEBUG sort trace
# usage: tools_r02_gpu.sh <tag> [pytest -k expr]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
K=${2:+-k "$2"}
echo "tests $(date)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread $K > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo "bench $(date)"
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "debug $(date)"
BZG_DEBUG=1 BZG_ONE_STREAM=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-h2h --no-extra > $O/debug.json 2> $O/debug.err || { echo "debug failed"; exit 1; }
echo "done $(date)"
