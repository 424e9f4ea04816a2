#!/bin/bash
# PMC passes (one counter group per rocprofv3 run; kernel-trace only, no sys/hip traces).
# usage: tools_pmc.sh <bytes> <outdir> "<set1>" "<set2>" ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
BYTES=$1; OUT=gpurun_out/$2; shift 2
mkdir -p $OUT
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python bench.py --bytes $BYTES --steps 1 --warmup 0 --no-cpu > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
