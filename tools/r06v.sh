#!/bin/bash
# Round-6 (development tool): same-box A/B of an env knob on the long-repeat text.
# usage: tools/r06v.sh <tag> VAR valA valB
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O; V=$2
for r in 1 2 3; do
  for val in $3 $4; do
    export $V=$val
    timeout -k 10 300 python tools/prof_config.py repeat 3 > $O/t_${val}_$r.log 2>&1 || { echo "repeat failed"; exit 1; }
    echo "$V=$val $(grep -E '^repeat ' $O/t_${val}_$r.log)"
  done
done
