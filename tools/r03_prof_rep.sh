#!/bin/bash
# kernel trace of one step of the long-repeat text variant (one stream)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra --repeat-frac 0.25 > $O/prof.log 2>&1 || { echo "trace failed"; tail -20 $O/prof.log; exit 1; }
echo "done $(date)"
