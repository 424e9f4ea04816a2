#!/bin/bash
# Round-6 (development tool): host-to-host pipeline over the batch pipeline -- its tests and
# h2h timings for several piece plans (BZG_H2H_PLAN, MB).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pipelined or host_path or chunked or outbuff" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for plan in default 200 100,300 128,384 150,350 100,200,300 64,192; do
  if [ $plan = default ]; then unset BZG_H2H_PLAN; else export BZG_H2H_PLAN=$plan; fi
  timeout -k 10 300 python tools/h2h_probe.py > $O/h2h_$plan.log 2>&1 || { echo "probe failed"; tail $O/h2h_$plan.log; exit 1; }
  echo "$plan: $(grep h2h $O/h2h_$plan.log | awk '{print $5}' | tr '\n' ' ')"
done
unset BZG_H2H_PLAN
BZG_H2H_DEBUG=1 BZG_H2H_PLAN=${2:-100,300} timeout -k 10 300 python tools/h2h_probe.py > $O/h2h_dbg.log 2>&1 || { echo "probe failed"; tail $O/h2h_dbg.log; exit 1; }
tail -25 $O/h2h_dbg.log
