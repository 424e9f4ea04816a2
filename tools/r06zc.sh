#!/bin/bash
# Round-6 (development tool): S3 doubling-loop changes -- BZG_CHECK on the long repeats, the
# deep-group / BWT GPU tests, long-repeat timing.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
BZG_CHECK=1 timeout -k 10 300 python tools/prof_config.py repeat 1 > $O/check_repeat.log 2>&1 || { echo "check failed"; tail -20 $O/check_repeat.log; exit 1; }
echo "check repeat: $(grep -c 'bzg check' $O/check_repeat.log) bad"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -k "deep or pair or doubling or periodic or bwt or long or round_trip" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 300 python tools/prof_config.py repeat 3 > $O/t_$r.log 2>&1 || { echo "repeat failed"; exit 1; }
  grep -E '^repeat ' $O/t_$r.log
done
