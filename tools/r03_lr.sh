#!/bin/bash
# long-repeat text diagnostics: BZG_DEBUG sort trace + kernel trace of one step (development tool)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
BZG_DEBUG=1 BZG_ONE_STREAM=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-h2h --no-extra --repeat-frac 0.25 > $O/dbg.json 2> $O/dbg.err || { echo "dbg failed"; tail -20 $O/dbg.err; exit 1; }
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra --repeat-frac 0.25 > $O/prof.log 2>&1 || { echo "trace failed"; tail -20 $O/prof.log; exit 1; }
python tools/trace_split.py $O/prof/run_kernel_trace.csv > $O/split.txt
if [ -n "$2" ]; then
  BZ2_AMD_LIB=$PWD/bzip2_amd/var/$2/libbz2_amd.so BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof2 -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof2.log 2>&1 || { echo "trace2 failed"; tail -20 $O/prof2.log; exit 1; }
  python tools/trace_split.py $O/prof2/run_kernel_trace.csv > $O/split2.txt
fi
echo "done $(date)"
