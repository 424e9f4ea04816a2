#!/bin/bash
# Round-6 (development tool): heap read-ahead variants (built by tools/variant.sh with -DBZG_HEAP_LA1 / LA2 /
# UP1 on the round's code before the shipped simplification): code-length parity, isolated heap latency
# probe and the text bench, same box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for v in la1u la1; do
  L=bzip2_amd/var/$v/libbz2_amd.so
  BZ2_AMD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "code_lengths or huff_spec or golden" > $O/t_$v.log 2>&1 || { echo "tests failed $v"; tail -20 $O/t_$v.log; exit 1; }
  echo "$v $(tail -1 $O/t_$v.log)"
  BZ2_AMD_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/h_$v -o run -- python tools/huff_probe.py > $O/h_$v.log 2>&1 || { echo "probe failed"; exit 1; }
done
for r in 1 2; do
  for v in la1u la1; do
    L=bzip2_amd/var/$v/libbz2_amd.so
    BZ2_AMD_LIB=$L timeout -k 10 200 python tools/small_probe.py > $O/s.log 2>&1 || { echo "probe failed"; tail $O/s.log; exit 1; }
    echo "$v $(tail -1 $O/s.log)"
    BZ2_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b.json 2> $O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  done
done
