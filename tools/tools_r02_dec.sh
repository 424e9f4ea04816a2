#!/bin/bash
# GPU decompression tests (tests/test_decomp.py) + smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decomp.py -m gpu -x -v --timeout 300 --timeout-method thread ${2:+-k "$2"} > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo "done $(date)"
