#!/bin/bash
# one GPU call: gpu tests, default bench, kernel-trace profile, HBM PMC passes (FETCH_SIZE / WRITE_SIZE)
# usage: tools_r01_gpu.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
echo "tests $(date)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo "bench $(date)"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "prof $(date)"
BZG_ONE_STREAM=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1)); echo "pmc $set $(date)"
  BZG_ONE_STREAM=1 timeout -k 10 400 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python bench.py --steps 1 --warmup 0 --no-cpu --no-h2h > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "done $(date)"
