#!/bin/bash
# Checkpoint: the whole GPU suite, smoke(), and the 2-rank torchrun rehearsal of the default bench.
set -o pipefail
mkdir -p gpurun_out/r3s
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3s/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3s/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3s/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s/smoke.log 2>&1 || { tail -20 gpurun_out/r3s/smoke.log; exit 1; }
tail -3 gpurun_out/r3s/smoke.log
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 1 --rehearse --no-host-path > gpurun_out/r3s/rehearse2.log 2>&1 || { tail -20 gpurun_out/r3s/rehearse2.log; exit 1; }
tail -1 gpurun_out/r3s/rehearse2.log | cut -c1-400
