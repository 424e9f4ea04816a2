#!/bin/bash
# Round-6 A/B on the text and the long-repeat text (development tool): variants "name:ENV=v,..."
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
envs() { [[ "$1" == *:* ]] && echo "${1#*:}" | tr ',' ' ' || echo ""; }
nm() { echo "${1%%:*}"; }
for r in 1 2; do
  for v in "$@"; do
    for k in text repeat; do
      env $(envs $v) timeout -k 10 300 python tools/prof_config.py $k 3 > $O/${k}_$(nm $v)_$r.log 2>&1 || { echo "failed: $v $k"; tail -20 $O/${k}_$(nm $v)_$r.log; exit 1; }
      echo "$(nm $v) $(grep MB/s $O/${k}_$(nm $v)_$r.log)"
    done
  done
done
echo "done $(date)"
