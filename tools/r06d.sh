#!/bin/bash
# Round-6 A/B of the wave-parallel Huffman heap (development tool): the code-length test for
# both builds, huff_probe kernel times, and the bench (text) for both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d; mkdir -p $O
SER=$PWD/bzip2_amd/var/heapser/libbz2_amd.so
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "code_lengths or golden or levels" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in par ser; do
  L=""; [ $v = ser ] && L=$SER
  env ${L:+BZ2_AMD_LIB=$L} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hp_$v -o run -- python tools/huff_probe.py > $O/hp_$v.log 2>&1 || { echo "probe failed $v"; tail -20 $O/hp_$v.log; exit 1; }
  python - "$O/hp_$v/run_kernel_trace.csv" <<'PY'
import csv,sys
rows=[r for r in csv.DictReader(open(sys.argv[1])) if 'code_lengths_test' in r['Kernel_Name']]
print(sys.argv[1].split('/')[-2], ' '.join(f"{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3:.0f}" for r in rows))
PY
done
for r in 1 2; do
  for v in par ser; do
    L=""; [ $v = ser ] && L=$SER
    env ${L:+BZ2_AMD_LIB=$L} timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-h2h --no-extra > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench failed"; tail $O/b_${v}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('stages_ms'))"
  done
done
for v in par ser; do
  L=""; [ $v = ser ] && L=$SER
  env ${L:+BZ2_AMD_LIB=$L} timeout -k 10 300 python tools/prof_config.py random 2 > $O/rnd_$v.log 2>&1 || { echo "random failed"; tail $O/rnd_$v.log; exit 1; }
  grep MB/s $O/rnd_$v.log
done
echo done
