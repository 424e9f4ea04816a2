#!/bin/bash
# GPU tests (optional -k filter), then a kernel trace of one workload of tools/prof_cfg.py
# usage: tools/r03_prof_cfg.sh <tag> <pytest -k expr | none> <text|random|single> [bytes] [steps]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
if [ "$2" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$2" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python tools/prof_cfg.py $3 ${4:-1000000000} ${5:-2} > $O/prof.log 2>&1 || { echo "trace failed"; tail -20 $O/prof.log; exit 1; }
grep "^step" $O/prof.log
python tools/trace_split.py $O/prof/run_kernel_trace.csv > $O/split.txt && head -40 $O/split.txt
echo "done $(date)"
