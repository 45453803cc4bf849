#!/bin/bash
# The driver's N > 1 launch shape, rehearsed with 2 ranks on the box's one GPU (--rehearse), on the
# final build: default weak bench, explicit --steps / --warmup as the driver passes them.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/final3e
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 20 --warmup 3 --rehearse --no-host-path > gpurun_out/final3e/rehearse2.log 2>&1 || { tail -20 gpurun_out/final3e/rehearse2.log; exit 1; }
tail -1 gpurun_out/final3e/rehearse2.log | cut -c1-500
