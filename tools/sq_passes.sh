#!/bin/bash
# SQ counter passes over one 1e9-byte text step (development tool), one-stream and production
# two-stream settings: issue split (active / stall / parked), instruction mix, LDS conflicts.
# With a second argument (single|random|repeat), one one-stream step of that tools/prof_config.py
# workload instead.
# usage: tools/sq_passes.sh <tag> [single|random|repeat]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; W=${2:-}; O=gpurun_out/$T; mkdir -p $O
CMD="python bench.py --steps 1 --warmup 0 --no-cpu --no-h2h --no-extra"
MODES="one two"
if [ -n "$W" ]; then CMD="python tools/prof_config.py $W 1"; MODES="one"; fi
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY"
S2="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"
for mode in $MODES; do
  i=0
  for set in "$S1" "$S2"; do
    i=$((i+1)); echo "pmc $mode $i $(date)"
    if [ $mode = one ]; then
      BZG_ONE_STREAM=1 timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $O/${mode}$i -o run -- $CMD > $O/${mode}$i.log 2>&1 || { echo "pass failed"; tail -20 $O/${mode}$i.log; exit 1; }
    else
      timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $O/${mode}$i -o run -- $CMD > $O/${mode}$i.log 2>&1 || { echo "pass failed"; tail -20 $O/${mode}$i.log; exit 1; }
    fi
  done
  python tools/sq_summary.py $O/${mode}1/run_counter_collection.csv 40 --tmpl --lds $O/${mode}2/run_counter_collection.csv > $O/sq_${mode}.txt
done
echo "done $(date)"
