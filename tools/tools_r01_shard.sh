#!/bin/bash
# GPU call: sharded-stream tests, then bench rehearsals (stream mode at N=1 on nccl, N=2 ranks on one GPU over gloo)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
echo "tests $(date)"
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "seg_walk or sharded or device_api" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo "bench stream N=1 $(date)"
timeout -k 10 300 python bench.py --mode stream --steps 3 --warmup 1 --no-cpu --no-h2h > $O/bench_s1.json 2> $O/bench_s1.err || { echo "bench s1 failed"; tail -20 $O/bench_s1.err; exit 1; }
cat $O/bench_s1.json
echo "bench stream N=2 gloo $(date)"
BZG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --bytes 300000000 --steps 2 --warmup 1 --no-cpu --no-h2h > $O/bench_s2.json 2> $O/bench_s2.err || { echo "bench s2 failed"; tail -30 $O/bench_s2.err; exit 1; }
cat $O/bench_s2.json
echo "done $(date)"
