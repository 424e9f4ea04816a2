set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-p100r6}; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python tools/gap_probe.py 100000000 > $O/probe.log 2>&1 && python tools/gap_probe.py --report $O/t/run_kernel_trace.csv > $O/report.txt
