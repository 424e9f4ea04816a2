#!/bin/bash
# parity subset + A/B bench lines over env variants (VARIANTS="A=1 B=2;C=3" ...)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-bwt or long_repeat or periodic or levels or golden or edge}" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
IFS=';' read -ra VS <<< "${VARIANTS:-BZG_S1P=0;BZG_S1P=1}"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-extra ${BENCHARGS} > $O/b$i.json 2> $O/b$i.err || { echo "bench failed: $v"; tail -5 $O/b$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$i.json'));print('$v', d['value'],d['stages_ms'])"
done
if [ -n "$TRACE" ]; then
  env $TRACE BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof.log 2>&1 || { echo "trace failed"; exit 1; }
fi
echo "done $(date)"
