#!/bin/bash
# Round-6 check of the S1 small-bucket finish (development tool): sort / stream GPU tests, then
# config 5 and the texts.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
BZG_CHECK=1 timeout -k 10 300 python tools/prof_config.py random 1 > $O/check.log 2>&1 || { echo "check failed"; tail -20 $O/check.log; exit 1; }
echo "check lines: $(grep -c 'bzg check' $O/check.log)"
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread -k "bwt or levels or golden or edge or random or periodic or quasi or mixed or repeats or deep" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for k in random text repeat; do
    timeout -k 10 300 python tools/prof_config.py $k 3 > $O/${k}_$r.log 2>&1 || { echo "failed $k"; tail -20 $O/${k}_$r.log; exit 1; }
    grep MB/s $O/${k}_$r.log
  done
done
echo "done $(date)"
