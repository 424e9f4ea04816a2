#!/bin/bash
# Same-box A/B on one tools/prof_config.py workload (development tool): 2 rounds over the
# variants, 3 steps each.  usage: tools/ab_config.sh <tag> <single|random|repeat> <variant>...
#   variant: "base" or a name under bzip2_amd/var/ (tools/variant.sh, tools/var_ref.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; K=$2; shift 2; O=gpurun_out/$T; mkdir -p $O
lib() { [ "$1" = base ] && echo "$PWD/bzip2_amd/libbz2_amd.so" || echo "$PWD/bzip2_amd/var/$1/libbz2_amd.so"; }
for r in 1 2; do
  for v in "$@"; do
    BZ2_AMD_LIB=$(lib $v) timeout -k 10 300 python tools/prof_config.py $K 3 > $O/cfg_${K}_${v}_$r.log 2>&1 || { echo "run failed: $v"; tail -20 $O/cfg_${K}_${v}_$r.log; exit 1; }
    echo "$v $(grep MB/s $O/cfg_${K}_${v}_$r.log)"
  done
done
echo "done $(date)"
