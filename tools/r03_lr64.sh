set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/lr64; mkdir -p $O
BZG_DWAVE_TINY=64 BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra --repeat-frac 0.25 > $O/prof.log 2>&1 || exit 1
python tools/trace_split.py $O/prof/run_kernel_trace.csv > $O/split.txt
