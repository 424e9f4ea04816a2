#!/bin/bash
# Round-6 (development tool): same-box A/B of the library before the Huffman round speculation
# ('pre') and with it ('cur'), plus cur with the speculation off (BZG_HUFF_SPEC_MAX=0).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for r in 1 2 3; do
  for v in pre cur cur0; do
    L=bzip2_amd/var/${v%0}/libbz2_amd.so; S=2048; [ $v = cur0 ] && S=0
    BZG_HUFF_SPEC_MAX=$S BZ2_AMD_LIB=$L timeout -k 10 200 python tools/small_probe.py > $O/s.log 2>&1 || { echo "probe failed"; tail $O/s.log; exit 1; }
    echo "$v $(tail -1 $O/s.log)"
    BZG_HUFF_SPEC_MAX=$S BZ2_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b.json 2> $O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  done
done
