#!/bin/bash
# Round-6 (development tool): h2h timings for piece plans given as arguments (BZG_H2H_PLAN, MB).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O; shift
for plan in "$@"; do
  if [ $plan = default ]; then unset BZG_H2H_PLAN; else export BZG_H2H_PLAN=$plan; fi
  timeout -k 10 300 python tools/h2h_probe.py > $O/h2h_$plan.log 2>&1 || { echo "probe failed"; tail $O/h2h_$plan.log; exit 1; }
  echo "$plan: $(grep '^h2h' $O/h2h_$plan.log | awk '{print $4}' | tr '\n' ' ')"
done
