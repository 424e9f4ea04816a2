#!/bin/bash
# PMC passes (one counter group per rocprofv3 run; kernel-trace only, no sys/hip traces).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python bench.py --bytes 100000000 --steps 1 --warmup 0 --no-cpu > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
