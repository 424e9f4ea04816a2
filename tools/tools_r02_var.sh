#!/bin/bash
# A/B bench lines over library variants: tools_r02_var.sh TAG default variants/a.so ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
i=0
for v in "$@"; do
  i=$((i+1))
  L=""; [ "$v" != default ] && L="$GRAFT_REPO_ROOT/$v"
  if [ -n "$VTEST" ]; then
    BZ2_AMD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "$VTEST" > $O/t$i.log 2>&1 || { echo "tests failed: $v"; tail -30 $O/t$i.log; exit 1; }
    echo "$v $(tail -1 $O/t$i.log)"
  fi
  BZ2_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-extra ${BENCHARGS} > $O/b$i.json 2> $O/b$i.err || { echo "bench failed: $v"; tail -5 $O/b$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$i.json'));print('$v', d['value'],d['stages_ms'])"
  if [ -n "$VTRACE" ]; then
    BZ2_AMD_LIB=$L BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof$i -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof$i.log 2>&1 || { echo "trace failed"; exit 1; }
    python3 tools_kstat_top.py $O/prof$i/run_kernel_stats.csv 12
  fi
done
echo "done $(date)"
