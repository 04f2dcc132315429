#!/bin/bash
# multi-rank rehearsal of bench.py on a 1-GPU box: 2 ranks share cuda:0 over gloo (RCCL needs one
# GPU per rank); small shards so both fit in one GPU's HBM
set -o pipefail
mkdir -p gpurun_out
PVAC_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --pairs 262144 \
  > gpurun_out/dist2.log 2>&1; rc=$?
grep '^{' gpurun_out/dist2.log | cut -c1-900; exit $rc
