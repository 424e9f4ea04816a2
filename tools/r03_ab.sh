#!/bin/bash
# Same-box A/B of library variants (development tool).
# usage: tools/r03_ab.sh <tag> <pytest -k expr | none> <variant> [variant ...]
#   variant: "base" (bzip2_amd/libbz2_amd.so) or a name under bzip2_amd/var/ (tools/variant.sh),
#   optionally with env settings: "notc:BZG_X=1"
# Runs the -k tests once per non-base variant, then benches the variants round-robin twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; K=$2; shift 2; O=gpurun_out/$T; mkdir -p $O
lib() { local v=${1%%:*}; [ "$v" = base ] && echo "$PWD/bzip2_amd/libbz2_amd.so" || echo "$PWD/bzip2_amd/var/$v/libbz2_amd.so"; }
envs() { [[ "$1" == *:* ]] && echo "${1#*:}" | tr ',' ' ' || echo ""; }
if [ "$K" != none ]; then
  for v in "$@"; do
    [ "${v%%:*}" = base ] && [[ "$v" != *:* ]] && continue
    echo "tests $v $(date)"
    env BZ2_AMD_LIB=$(lib $v) $(envs $v) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests_${v%%:*}.log 2>&1 || { echo "tests failed: $v"; tail -30 $O/tests_${v%%:*}.log; exit 1; }
    tail -1 $O/tests_${v%%:*}.log
  done
fi
for r in 1 2; do
  for v in "$@"; do
    n=$(echo "$v" | tr ':=,/' '____')
    env BZ2_AMD_LIB=$(lib $v) $(envs $v) timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b_${n}_$r.json 2> $O/b_${n}_$r.err || { echo "bench failed: $v"; tail -20 $O/b_${n}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${n}_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  done
done
echo "done $(date)"
