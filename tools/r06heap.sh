#!/bin/bash
# Round-6 (development tool): the simplified heap -- parity subset, k_huff_spec on / off on the small
# probe, and config 5 with k_huff_lanes (default) against the single-lane heap everywhere.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "code_lengths or golden or levels or pipelined or full_size or huff_spec or split_batches" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 512 0; do
    BZG_HUFF_SPEC_MAX=$v timeout -k 10 200 python tools/small_probe.py > $O/s.log 2>&1 || { echo "probe failed"; tail $O/s.log; exit 1; }
    echo "spec_max=$v $(tail -1 $O/s.log)"
  done
done
for v in 4096 1000000000; do
  BZG_HUFF_LANES_MIN=$v BZG_BATCH_PIPE=0 timeout -k 10 300 python tools/prof_config.py random 2 > $O/r.log 2>&1 || { echo "random failed"; tail $O/r.log; exit 1; }
  echo "lanes_min=$v $(grep -E '^random ' $O/r.log | tail -1)"
done
