#!/bin/bash
# quick parity subset, one bench line, then PMC passes (tools_r02_pmc.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "${TESTK:-bwt or golden or levels or edge}" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-extra > $O/b.json 2> $O/b.err || { echo "bench failed"; tail -5 $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['stages_ms'])"
[ $# -gt 0 ] && ./tools_r02_pmc.sh $T/pmc "$@"
echo "done $(date)"
