#!/bin/bash
# Round-6 (development tool): k_huff_spec threshold 512 against 1024 with the simplified heap (the
# strong shares of bench.py: 250 MB = 834 tables per launch).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for v in 512 1024 512 1024; do
  BZG_HUFF_SPEC_MAX=$v timeout -k 10 600 python bench.py --no-cpu --no-h2h > $O/b.json 2> $O/b.err || { echo "bench failed"; tail -20 $O/b.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/b.json'));s=d['secondary']
print('spec_max=$v', d['value'], d['ms_per_step'], d['stages_ms']['code'], 'enwik8', s['enwik8_100mb']['ms_per_step'], s['enwik8_100mb']['stages_ms']['code'], {k:(v['ms'],v['stages_ms']['code']) for k,v in s['strong_shares']['shares'].items()})"
done
