#!/bin/bash
# Round-4 same-box A/B (development tool): optional -k GPU tests per variant, then the bench
# round-robin over the variants (3 rounds), then a one-stream kernel trace per variant.
# usage: tools/ab.sh <tag> <pytest -k expr | none> <variant> [variant ...]
#   variant: "base" or a name under bzip2_amd/var/ (tools/variant.sh), optionally ":ENV=1,ENV2=2"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; K=$2; shift 2; O=gpurun_out/$T; mkdir -p $O
lib() { local v=${1%%:*}; [ "$v" = base ] && echo "$PWD/bzip2_amd/libbz2_amd.so" || echo "$PWD/bzip2_amd/var/$v/libbz2_amd.so"; }
envs() { [[ "$1" == *:* ]] && echo "${1#*:}" | tr ',' ' ' || echo ""; }
nm() { echo "$1" | tr ':=,/' '____'; }
if [ "$K" != none ]; then
  for v in "$@"; do
    echo "tests $v $(date)"
    env BZ2_AMD_LIB=$(lib $v) $(envs $v) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests_$(nm $v).log 2>&1 || { echo "tests failed: $v"; tail -30 $O/tests_$(nm $v).log; exit 1; }
    tail -1 $O/tests_$(nm $v).log
  done
fi
for r in 1 2 3; do
  for v in "$@"; do
    env BZ2_AMD_LIB=$(lib $v) $(envs $v) timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b_$(nm $v)_$r.json 2> $O/b_$(nm $v)_$r.err || { echo "bench failed: $v"; tail -20 $O/b_$(nm $v)_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_$(nm $v)_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  done
done
for v in "$@"; do
  env BZ2_AMD_LIB=$(lib $v) $(envs $v) BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$(nm $v) -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof_$(nm $v).log 2>&1 || { echo "trace failed: $v"; tail -20 $O/prof_$(nm $v).log; exit 1; }
  python tools/trace_split.py $O/prof_$(nm $v)/run_kernel_trace.csv > $O/split_$(nm $v).txt
done
echo "done $(date)"
