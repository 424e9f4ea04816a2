#!/bin/bash
# one GPU call: gpu tests (optional -k filter), then the default bench line
# usage: tools/r03_gpu.sh <tag> [pytest -k expr] [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
K=()
[ -n "$2" ] && K=(-k "$2")
shift; shift
echo "tests $(date)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread "${K[@]}" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
if [ "$1" != "nobench" ]; then
  echo "bench $(date)"
  timeout -k 10 600 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
echo "done $(date)"
