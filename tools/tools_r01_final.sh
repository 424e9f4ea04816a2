#!/bin/bash
# GPU call: full gpu tests, default bench, stream-mode bench with per-step timing, kernel-trace profile of the stream mode
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
echo "tests $(date)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo "bench $(date)"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "bench stream $(date)"
BZG_SHARD_TIMING=1 timeout -k 10 300 python bench.py --mode stream --steps 3 --warmup 1 --no-cpu --no-h2h > $O/bench_stream.json 2> $O/bench_stream.err || { echo "bench stream failed"; exit 1; }
cat $O/bench_stream.json
echo "prof stream $(date)"
BZG_ONE_STREAM=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_stream -o run -- python bench.py --mode stream --steps 1 --warmup 1 --no-cpu --no-h2h > $O/prof_stream.log 2>&1 || { echo "prof failed"; exit 1; }
echo "done $(date)"
