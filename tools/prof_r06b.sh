#!/bin/bash
# Round-6 kernel traces (development tool): decode of the text stream, config 5, long repeats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
echo "decode $(date)"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_dec -o run -- python tools/prof_config.py text 1 decode > $O/prof_dec.log 2>&1 || { echo "trace dec failed"; tail -20 $O/prof_dec.log; exit 1; }
grep -E "decode|MB/s" $O/prof_dec.log
bash tools/prof_configs.sh $T random repeat
