#!/bin/bash
# 2-rank stream-mode rehearsal of bench.py on the box's one GPU over gloo (not a perf figure)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
echo "dist $(date)"
BZG_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --bytes 200000000 --no-cpu --no-h2h > $O/dist.json 2> $O/dist.err || { echo "dist failed"; tail -30 $O/dist.err; exit 1; }
cat $O/dist.json
echo "done $(date)"
