#!/bin/bash
# Round-6 (development tool): small-call timings against the parts per batch (BZG_PARTS) and
# the split table streams (BZG_SPLIT_TABLES), same box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  for v in "BZG_PARTS=2" "BZG_PARTS=1" "BZG_PARTS=4" "BZG_SPLIT_TABLES=0"; do
    env $v timeout -k 10 200 python tools/small_probe.py > $O/s.log 2>&1 || { echo "probe failed"; tail $O/s.log; exit 1; }
    echo "$v $(tail -1 $O/s.log)"
  done
done
