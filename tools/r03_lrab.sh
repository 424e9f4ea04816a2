#!/bin/bash
# long-repeat A/B over env settings (development tool): tools/r03_lrab.sh <tag> <pytest -k|none> "<ENV=..>" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; K=$2; shift 2; O=gpurun_out/$T; mkdir -p $O
if [ "$K" != none ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-extra --repeat-frac 0.25 > $O/b$i.json 2> $O/b$i.err || { echo "bench $i failed"; tail -20 $O/b$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d.get('stages_ms'))"
done
echo "done $(date)"
