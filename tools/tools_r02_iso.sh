#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/iso; mkdir -p $O
for v in "BZG_S1P=1" "BZG_S1P=1 BZG_FULL_UNIT_OUT=1" "BZG_S1P=0" "BZG_S1P=0 BZG_FULL_UNIT_OUT=1"; do
  echo "== $v"
  env $v timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread -k "many_deep" > $O/t.log 2>&1; echo "rc=$?"; tail -1 $O/t.log
done
