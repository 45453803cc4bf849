#!/bin/bash
# C5 rehearsal: 2 ranks under torchrun on the box's one GPU (--rehearse), weak and strong modes
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --rehearse > gpurun_out/rehearse_weak.log 2>&1 || exit 1
tail -1 gpurun_out/rehearse_weak.log | cut -c1-300
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --scaling strong --total-pairs 4000000 --steps 2 --warmup 1 --rehearse > gpurun_out/rehearse_strong.log 2>&1 || exit 1
tail -1 gpurun_out/rehearse_strong.log | cut -c1-300
