#!/bin/bash
# Round-6 (development tool): branch-free DOWNHEAP A/B (BZG_HEAP_BF) -- Huffman test-kernel
# latencies, the Huffman / stream GPU tests, text bench, small probe, config 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for v in 0 1; do
  BZG_HEAP_BF=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/hp_$v -o run -- python3 tools/huff_probe.py > $O/hp_$v.log 2>&1 || { echo "probe failed"; tail $O/hp_$v.log; exit 1; }
  f=$(find $O/hp_$v -name '*kernel_trace.csv' | head -1)
  echo "bf=$v us: $(python3 -c "
import csv,sys
r=[x for x in csv.DictReader(open('$f')) if 'k_code_lengths_test' in x['Kernel_Name']]
r.sort(key=lambda x:int(x['Start_Timestamp']))
print(' '.join(str((int(x['End_Timestamp'])-int(x['Start_Timestamp']))//1000) for x in r))")"
done
BZG_HEAP_BF=1 timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "code_lengths or huffman or golden or levels" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/r06u.sh $1_ab BZG_HEAP_BF 0 1
for v in 0 1; do
  BZG_HEAP_BF=$v timeout -k 10 300 python tools/prof_config.py random 2 > $O/r_$v.log 2>&1 || { echo "random failed"; exit 1; }
  echo "bf=$v $(grep -E '^random ' $O/r_$v.log)"
done
