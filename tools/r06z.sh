#!/bin/bash
# Round-6 (development tool): same-box A/B of two library builds (BZ2_AMD_LIB) on the text
# bench, the small probe and long repeats.  usage: tools/r06z.sh <tag> <varA> <varB>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for r in 1 2 3; do
  for v in $2 $3; do
    BZ2_AMD_LIB=bzip2_amd/var/$v/libbz2_amd.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench failed"; tail $O/b_${v}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  done
done
for v in $2 $3; do
  BZ2_AMD_LIB=bzip2_amd/var/$v/libbz2_amd.so timeout -k 10 300 python tools/small_probe.py > $O/s_$v.log 2>&1 || { echo "probe failed"; exit 1; }
  echo "$v $(tail -1 $O/s_$v.log)"
  BZ2_AMD_LIB=bzip2_amd/var/$v/libbz2_amd.so timeout -k 10 300 python tools/prof_config.py repeat 2 > $O/t_$v.log 2>&1 || { echo "repeat failed"; exit 1; }
  echo "$v $(grep -E '^repeat ' $O/t_$v.log)"
done
