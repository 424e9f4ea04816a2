#!/bin/bash
# S2->S3 handoff depth sweep on plain and long-repeat text (bench lines only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
for rf in 0 0.25; do
  for dw in ${DWAVES:-1024 256 128 64}; do
    BZG_DWAVE=$dw timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-h2h --no-extra --repeat-frac $rf > $O/b_${rf}_$dw.json 2> $O/b_${rf}_$dw.err || { echo "bench failed $rf $dw"; tail -5 $O/b_${rf}_$dw.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_${rf}_$dw.json'));print('rf $rf dwave $dw', d['value'],d['stages_ms'])"
  done
done
echo "done $(date)"
