#!/bin/bash
# kernel-trace profile of one bench step at the given size: tools_prof.sh <bytes> <outdir>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
BZG_ONE_STREAM=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/$2 -o run -- python bench.py --bytes $1 --steps 1 --warmup 1 --no-cpu > gpurun_out/$2.log 2>&1
