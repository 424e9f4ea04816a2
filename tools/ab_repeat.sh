#!/bin/bash
# Same-box A/B of the bench text and the long-repeat text (development tool).
# usage: tools/ab_repeat.sh <tag> <pytest -k expr | none> <variant> [variant ...]
#   variant: "base" or a name under bzip2_amd/var/ (tools/variant.sh), optionally ":ENV=1,ENV2=2"
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; K=$2; shift 2; O=gpurun_out/$T; mkdir -p $O
lib() { local v=${1%%:*}; [ "$v" = base ] && echo "$PWD/bzip2_amd/libbz2_amd.so" || echo "$PWD/bzip2_amd/var/$v/libbz2_amd.so"; }
envs() { [[ "$1" == *:* ]] && echo "${1#*:}" | tr ',' ' ' || echo ""; }
nm() { echo "$1" | tr ':=,/' '____'; }
if [ "$K" != none ]; then
  for v in "$@"; do
    env BZ2_AMD_LIB=$(lib $v) $(envs $v) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests_$(nm $v).log 2>&1 || { echo "tests failed: $v"; tail -30 $O/tests_$(nm $v).log; exit 1; }
    echo "tests $v: $(tail -1 $O/tests_$(nm $v).log)"
  done
fi
for r in 1 2; do
  for v in "$@"; do
    env BZ2_AMD_LIB=$(lib $v) $(envs $v) timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b_$(nm $v)_$r.json 2> $O/b_$(nm $v)_$r.err || { echo "bench failed: $v"; tail -20 $O/b_$(nm $v)_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_$(nm $v)_$r.json').read().strip().splitlines()[-1]); print('$v text', d['value'], d['ms_per_step'], d.get('stages_ms'))"
    env BZ2_AMD_LIB=$(lib $v) $(envs $v) timeout -k 10 300 python tools/prof_config.py repeat 3 > $O/r_$(nm $v)_$r.log 2>&1 || { echo "repeat failed: $v"; tail -20 $O/r_$(nm $v)_$r.log; exit 1; }
    echo "$v $(grep MB/s $O/r_$(nm $v)_$r.log)"
  done
done
echo "done $(date)"
