#!/bin/bash
# Round-6 (development tool): lane-per-table Huffman (k_huff_lanes) -- parity through the
# code-length hook and whole streams with it forced (BZG_HUFF_LANES_MIN=0), then timings of
# the text bench, small calls and config 5 for never / default / always.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
BZG_HUFF_LANES_MIN=0 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -k "code_length or huffman or golden or levels or stream or round_trip or full_size or split_batches" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1000000000 4096 0; do
    BZG_HUFF_LANES_MIN=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench failed"; tail $O/b_${v}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('min=$v', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  done
done
for v in 1000000000 4096 0; do
  BZG_HUFF_LANES_MIN=$v timeout -k 10 300 python tools/small_probe.py > $O/s_$v.log 2>&1 || { echo "probe failed"; exit 1; }
  echo "min=$v $(tail -1 $O/s_$v.log)"
  BZG_HUFF_LANES_MIN=$v BZG_BATCH_PIPE=0 timeout -k 10 300 python tools/prof_config.py random 2 > $O/r_$v.log 2>&1 || { echo "random failed"; exit 1; }
  echo "min=$v seq $(grep -E '^random ' $O/r_$v.log)"
done
