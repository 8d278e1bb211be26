#!/bin/bash
# The N > 1 bench flow rehearsed on one GPU: two ranks under torch.distributed.run with the gloo backend
# (partials gathered through host memory; the driver's multi-GPU runs use RCCL), for every workload.
cd "$(dirname "$0")/../.." || exit 1
export DDSHE_DIST_BACKEND=gloo
R="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
tools/gpurun/steps.sh \
  "400 d2 $R --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1" \
  "300 d2o $R --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --workload order" \
  "300 d2e $R --master-port 29513 bench.py --gpus 2 --steps 3 --warmup 1 --workload entry_search" \
  "300 d2p $R --master-port 29514 bench.py --gpus 2 --steps 3 --warmup 1 --workload product_filter" \
  "400 d2c $R --master-port 29515 bench.py --gpus 2 --steps 1 --warmup 0 --workload encrypt_sum"
