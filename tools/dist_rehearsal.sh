#!/bin/bash
# 2-rank stream-mode rehearsals of `bench.py --gpus 2` on the box's one GPU over gloo: bench.py
# launches its two ranks itself (not a perf figure; both ranks share the GPU).  First weak
# scaling (200 MB per rank), then BASELINE config 3 as stated (--total-bytes 1e9: one stream of
# 1e9 B split over the ranks).
# usage: tools/dist_rehearsal.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
echo "dist weak $(date)"
BZG_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 2 --warmup 1 --bytes 200000000 --no-cpu --no-h2h > $O/dist.json 2> $O/dist.err || { echo "dist failed"; tail -30 $O/dist.err; exit 1; }
cat $O/dist.json
echo "dist strong $(date)"
BZG_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 2 --warmup 1 --total-bytes 1000000000 --no-cpu --no-extra > $O/dist_strong.json 2> $O/dist_strong.err || { echo "dist strong failed"; tail -30 $O/dist_strong.err; exit 1; }
cat $O/dist_strong.json
echo "done $(date)"
