#!/bin/bash
# PMC passes over one 1e9-byte step (kernel trace + one counter set per rocprofv3 run).
# usage: tools/pmc_passes.sh <tag> "<set1>" "<set2>" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
BYTES=${BZG_PMC_BYTES:-1000000000}
echo "trace $(date)"
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --bytes $BYTES --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof.log 2>&1 || { echo "trace failed"; tail -20 $O/prof.log; exit 1; }
i=0
for set in "$@"; do
  i=$((i+1)); echo "pmc $set $(date)"
  BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python bench.py --bytes $BYTES --steps 1 --warmup 0 --no-cpu --no-h2h --no-extra > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $O/p$i.log; exit 1; }
done
echo "done $(date)"
