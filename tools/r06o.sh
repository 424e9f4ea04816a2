#!/bin/bash
# Round-6 small-call trace (development tool): one 100 MB call's kernel timeline and gaps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/gap_probe.py ${2:-100000000} > $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
cat $O/probe.log | grep call
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python tools/gap_probe.py --report $f > $O/gaps.txt && head -30 $O/gaps.txt
python tools/trace_split.py $f > $O/split.txt && head -60 $O/split.txt
