#!/bin/bash
# Round-6 (development tool): k_cf / k_pack workgroups per block (BZG_SLICE_MAX, BZG_SLICE_FILL)
# on the small probe and the text bench, same box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  for v in "8 768" "16 1536" "16 768" "32 3072"; do
    set -- $v
    BZG_SLICE_MAX=$1 BZG_SLICE_FILL=$2 timeout -k 10 200 python tools/small_probe.py > $O/s.log 2>&1 || { echo "probe failed"; tail $O/s.log; exit 1; }
    echo "max=$1 fill=$2 $(tail -1 $O/s.log)"
  done
done
for v in "8 768" "16 1536"; do
  set -- $v
  BZG_SLICE_MAX=$1 BZG_SLICE_FILL=$2 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b.json 2> $O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('max=$1 fill=$2', d['value'], d['ms_per_step'], d.get('stages_ms'))"
done
