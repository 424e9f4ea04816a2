#!/bin/bash
# Round-6 decode trace (development tool).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_dec -o run -- python tools/prof_config.py text 1 decode > $O/prof_dec.log 2>&1 || { echo "trace dec failed"; tail -20 $O/prof_dec.log; exit 1; }
grep -E "decode|MB/s" $O/prof_dec.log
echo done
