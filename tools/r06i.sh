#!/bin/bash
# Round-6 cross-batch pipeline check (development tool): the multi-batch GPU tests, then
# config 5 and config 4 with the pipeline on and off, then the bench text line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread -k "pipelined_batches or full_size or split_batches or continuation or round_trip_large or host_pipelined or multi_device or golden" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    BZG_BATCH_PIPE=$v timeout -k 10 300 python tools/prof_config.py random 3 > $O/rnd_${v}_$r.log 2>&1 || { echo "random failed"; tail $O/rnd_${v}_$r.log; exit 1; }
    echo "pipe=$v $(grep MB/s $O/rnd_${v}_$r.log)"
  done
done
for v in 1 0; do
  BZG_BATCH_PIPE=$v timeout -k 10 300 python tools/prof_config.py single 3 > $O/one_${v}.log 2>&1 || { echo "single failed"; tail $O/one_${v}.log; exit 1; }
  echo "pipe=$v $(grep MB/s $O/one_${v}.log)"
done
echo "done $(date)"
