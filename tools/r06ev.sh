#!/bin/bash
# Round-6 (development tool): parity subset and the small probe after a host-side change.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "golden or levels or pipelined or full_size or huff_spec or split_batches or continuation or threads" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 200 python tools/small_probe.py > $O/s.log 2>&1 || { echo "probe failed"; tail $O/s.log; exit 1; }
  tail -1 $O/s.log
done
