#!/bin/bash
# Round-6 (development tool): sort pass structure of a 100 MB call (BZG_DEBUG counters).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
BZG_DEBUG=1 timeout -k 10 300 python3 tools/gap_probe.py ${2:-100000000} > $O/debug.log 2>&1 || { echo "probe failed"; tail -20 $O/debug.log; exit 1; }
grep -c "" $O/debug.log
