#!/bin/bash
# Round-3 final measurement on one GPU (development tool): full GPU tests, the default bench
# line, a kernel trace of one text step, and the FETCH_SIZE / WRITE_SIZE passes.
# usage: tools/final.sh <tag> [tests|notests]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
if [ "$2" != notests ]; then
  echo "tests $(date)"
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
echo "bench $(date)"
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "trace $(date)"
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof.log 2>&1 || { echo "trace failed"; tail -20 $O/prof.log; exit 1; }
python tools/trace_split.py $O/prof/run_kernel_trace.csv > $O/split.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof2 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof2.log 2>&1 || { echo "trace2 failed"; tail -20 $O/prof2.log; exit 1; }
echo "pmc $(date)"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python bench.py --steps 1 --warmup 0 --no-cpu --no-h2h --no-extra > $O/p$i.log 2>&1 || { echo "pmc $set failed"; tail -20 $O/p$i.log; exit 1; }
done
echo "done $(date)"
