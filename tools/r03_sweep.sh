#!/bin/bash
# bench the main workload under several BZG_* settings (same box, back to back)
# usage: tools/r03_sweep.sh <tag> "<ENV=.. ENV=..>" ["<...>" ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i+1))
  echo "cfg $i: $cfg $(date)"
  env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b$i.json 2> $O/b$i.err || { echo "bench $i failed"; tail -20 $O/b$i.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d.get('stages_ms'))"
done
echo "done $(date)"
