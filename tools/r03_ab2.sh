#!/bin/bash
# text + long-repeat A/B of library variants (development tool): tools/r03_ab2.sh <tag> <variant>...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
lib() { [ "$1" = base ] && echo "$PWD/bzip2_amd/libbz2_amd.so" || echo "$PWD/bzip2_amd/var/$1/libbz2_amd.so"; }
for r in 1 2; do
  for v in "$@"; do
    for w in text rep; do
      RF=0; [ $w = rep ] && RF=0.25
      BZ2_AMD_LIB=$(lib $v) timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-extra --repeat-frac $RF > $O/b_${v}_${w}_$r.json 2> $O/b_${v}_${w}_$r.err || { echo "bench failed: $v $w"; tail -20 $O/b_${v}_${w}_$r.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/b_${v}_${w}_$r.json').read().strip().splitlines()[-1]); print('$v $w', d['value'], d['ms_per_step'], d.get('stages_ms'))"
    done
  done
done
echo "done $(date)"
