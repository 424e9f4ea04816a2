#!/bin/bash
# Round-6 (development tool): A5 / periodic / multi-batch GPU tests and the default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -k "periodic or pipelined or copy_rank or single_byte or root or full_size or split_batches" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python - <<PY
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d.get('stages_ms'))
print('h2h', d['host_to_host'])
for k,v in d['secondary'].items():
    if 'value' in v: print(k, v['value'], v.get('ms_per_step'), v.get('stages_ms'), v.get('sequential'))
print(d['secondary']['strong_shares'])
PY
