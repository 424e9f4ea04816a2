#!/bin/bash
# Round-6 (development tool): k_huff_spec at up to 512 tables per launch -- parity tests and the
# default bench line (strong shares).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "code_lengths or golden or levels or pipelined_batches" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "
import json;d=json.load(open('$O/bench.json'));s=d['secondary']
print(d['value'], d['ms_per_step'], d['stages_ms'])
print('enwik8', s['enwik8_100mb']['value'], s['enwik8_100mb']['ms_per_step'], s['enwik8_100mb']['stages_ms'])
print({k:(v['ms'],v['ms_per_gb_vs_1gb'],v['stages_ms']['code']) for k,v in s['strong_shares']['shares'].items()})"
