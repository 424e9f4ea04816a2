#!/bin/bash
# Round-6 decode check (development tool): decompression tests, the 4 GiB PRNG round trip, and
# the decode timing of the 1 GB text stream.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_decomp.py tests/test_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread -k "decomp or decode or full_size_random or magics or golden" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/prof_config.py text 3 decode > $O/dec.log 2>&1 || { echo "dec failed"; tail -20 $O/dec.log; exit 1; }
grep -E "decode|MB/s" $O/dec.log
echo "done $(date)"
