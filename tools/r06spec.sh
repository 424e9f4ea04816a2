#!/bin/bash
# Round-6 (development tool): Huffman rounds 1 and 2 at once (BZG_HUFF_SPEC_MAX = tables per
# launch up to which k_huff runs two waves per table; 0 = never) -- parity tests, then the
# small probe and the text bench per setting, same box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "code_lengths or golden or levels or pipelined_batches or full_size" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 2048 0 8192; do
    BZG_HUFF_SPEC_MAX=$v timeout -k 10 200 python tools/small_probe.py > $O/s.log 2>&1 || { echo "probe failed"; tail $O/s.log; exit 1; }
    echo "spec_max=$v $(tail -1 $O/s.log)"
    BZG_HUFF_SPEC_MAX=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b.json 2> $O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('spec_max=$v', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  done
done
