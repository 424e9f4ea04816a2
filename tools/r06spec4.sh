#!/bin/bash
# Round-6 (development tool): k_huff_spec launch times per variant (kernel trace of the small
# probe): cur, nofence (fences dropped: timing only), r2idle (round-2 workgroups idle), and
# cur with the speculation off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for v in cur nofence r2idle cur0; do
  L=bzip2_amd/var/${v%0}/libbz2_amd.so; S=2048; [ $v = cur0 ] && S=0
  BZG_HUFF_SPEC_MAX=$S BZ2_AMD_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python tools/small_probe.py > $O/$v.log 2>&1 || { echo "$v failed"; tail $O/$v.log; exit 1; }
  echo "$v $(grep 100MB $O/$v.log | tail -1)"
  grep -E "k_huff" $O/$v/run_kernel_stats.csv | cut -d, -f1-6
done
