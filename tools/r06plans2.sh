#!/bin/bash
# Round-6 (development tool): host-to-host piece plans (BZG_H2H_PLAN) with the final code, same box, two rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  for v in default 64,256,400 100,300,500 80,240,480 50,200,400; do
    if [ $v = default ]; then unset BZG_H2H_PLAN; else export BZG_H2H_PLAN=$v; fi
    timeout -k 10 200 python tools/h2h_probe.py > $O/h.log 2>&1 || { echo "probe failed"; tail $O/h.log; exit 1; }
    echo "$v: $(grep '^h2h' $O/h.log | awk '{printf "%s ", $4}')"
  done
done
