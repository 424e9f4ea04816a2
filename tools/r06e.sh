#!/bin/bash
# Round-6 environment-knob A/B (development tool): 1e9 B bench text and 100 MB calls, per
# variant "name:ENV=v,ENV2=w" (base = no settings), two rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
envs() { [[ "$1" == *:* ]] && echo "${1#*:}" | tr ',' ' ' || echo ""; }
nm() { echo "${1%%:*}"; }
for r in 1 2; do
  for v in "$@"; do
    env $(envs $v) timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b_$(nm $v)_$r.json 2> $O/b_$(nm $v)_$r.err || { echo "bench failed: $v"; tail -20 $O/b_$(nm $v)_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_$(nm $v)_$r.json').read().strip().splitlines()[-1]); print('$(nm $v) 1e9', d['value'], d['ms_per_step'], d.get('stages_ms'))"
    env $(envs $v) timeout -k 10 300 python tools/small_probe.py > $O/s_$(nm $v)_$r.log 2>&1 || { echo "probe failed: $v"; tail -20 $O/s_$(nm $v)_$r.log; exit 1; }
    echo "$(nm $v) $(tail -1 $O/s_$(nm $v)_$r.log)"
  done
done
echo "done $(date)"
