#!/bin/bash
# Round-6 (development tool): correctness of a library variant (BZG_CHECK runs, sort / stream
# GPU tests through BZ2_AMD_LIB), then the same-box A/B of tools/r06z.sh.
# usage: tools/r06za.sh <tag> <base> <variant>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
export BZ2_AMD_LIB=bzip2_amd/var/$3/libbz2_amd.so
for k in text repeat random; do
  BZG_CHECK=1 timeout -k 10 300 python tools/prof_config.py $k 1 > $O/check_$k.log 2>&1 || { echo "check $k failed"; tail -20 $O/check_$k.log; exit 1; }
  echo "check $k: $(grep -c 'bzg check' $O/check_$k.log) bad"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -k "bwt or sort or golden or levels or periodic or deep or stream or round_trip or edge" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
unset BZ2_AMD_LIB
bash tools/r06z.sh $1 $2 $3
