#!/bin/bash
# k_s1p vs k_s1s: parity tests, bench lines, debug traces
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bwt or long_repeat or periodic or levels or golden or edge or round_trip" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for s1p in 1 0; do
  for rf in 0 0.25; do
    echo "s1p $s1p rf $rf $(date)"
    BZG_S1P=$s1p timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-extra --repeat-frac $rf > $O/b_${s1p}_${rf}.json 2> $O/b_${s1p}_${rf}.err || { echo "bench failed"; tail -5 $O/b_${s1p}_${rf}.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_${s1p}_${rf}.json'));print(d['value'],d['stages_ms'])"
  done
done
BZG_DEBUG=1 BZG_ONE_STREAM=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-h2h --no-extra > $O/debug.json 2> $O/debug.err || exit 1
BZG_DEBUG=1 BZG_ONE_STREAM=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-h2h --no-extra --repeat-frac 0.25 > $O/debug_rep.json 2> $O/debug_rep.err || exit 1
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof.log 2>&1 || { echo "trace failed"; exit 1; }
echo "done $(date)"
