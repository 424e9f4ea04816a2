#!/bin/bash
# Round-6 measurement on one GPU (development tool): optional GPU tests, the default bench line
# (with its secondary lines), and kernel traces of small calls (tools/gap_probe.py).
# usage: tools/r06.sh <tag> [tests|notests] [bench|nobench] [env settings for the probes...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
shift
TESTS=${1:-tests}; shift
BENCH=${1:-bench}; shift
if [ "$TESTS" = tests ]; then
  echo "tests $(date)"
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
if [ "$BENCH" = bench ]; then
  echo "bench $(date)"
  timeout -k 10 1000 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
for n in 100000000 1000000000; do
  echo "probe $n $(date)"
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p$n -o run -- python tools/gap_probe.py $n > $O/p$n.log 2>&1 || { echo "probe failed"; tail -20 $O/p$n.log; exit 1; }
  cat $O/p$n.log | grep call
  python tools/gap_probe.py --report $O/p$n/run_kernel_trace.csv | head -3
done
echo "done $(date)"
