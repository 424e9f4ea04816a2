#!/bin/bash
# Round-6 (development tool): the 1 GB text bench cut into pipelined batches (BZG_MAX_BATCH)
# against one batch, same box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  for v in 1500000000 500000000 700000000 350000000; do
    BZG_MAX_BATCH=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b.json 2> $O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('max_batch=$v', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  done
done
