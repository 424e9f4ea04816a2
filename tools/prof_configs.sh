#!/bin/bash
# Kernel traces of BASELINE configs 4 and 5 and of the long-repeat text (development tool); one
# sort stream and the batches one after another, so that kernel durations do not overlap.
# usage: tools/prof_configs.sh <tag> [single] [random] [repeat]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
for k in "$@"; do
  echo "$k $(date)"
  BZG_ONE_STREAM=1 BZG_BATCH_PIPE=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$k -o run -- python tools/prof_config.py $k 2 > $O/prof_$k.log 2>&1 || { echo "trace $k failed"; tail -20 $O/prof_$k.log; exit 1; }
  grep -E "MB/s" $O/prof_$k.log
  python tools/trace_split.py $O/prof_$k/run_kernel_trace.csv > $O/split_$k.txt
done
echo "done $(date)"
