#!/bin/bash
# decoder kernel profile (1e9 text) + full default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/dprof -o run -- python tools_decprof.py 1000000000 2 > $O/dprof.log 2>&1 || { echo "dprof failed"; tail -20 $O/dprof.log; exit 1; }
grep rep $O/dprof.log
if [ "$2" != "nobench" ]; then
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
fi
echo "done $(date)"
