#!/bin/bash
# kernel-trace profile of one 1e9-byte text step (one stream), plus a BZG_DEBUG trace of the
# config-4 tail sort.  usage: tools/r03_prof.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
BZG_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --no-cpu --no-h2h --no-extra > $O/prof.log 2>&1 || { echo "trace failed"; tail -20 $O/prof.log; exit 1; }
BZG_DEBUG=1 BZG_ONE_STREAM=1 timeout -k 10 300 python -c "
import torch, bzip2_amd as B, time
n = 4 * 2**30
d = torch.full((n,), 0x61, dtype=torch.uint8, device='cuda')
cap = B.bound(n); o = torch.empty(cap, dtype=torch.uint8, device='cuda')
for i in range(2):
    nb, _, _ = B.compress_device(d.data_ptr(), n, 9, o.data_ptr(), cap)
    torch.cuda.synchronize()
    print('config4', nb, B.last_stats(), flush=True)
" > $O/c4.log 2>&1 || { echo "c4 failed"; tail -20 $O/c4.log; exit 1; }
echo "done $(date)"
