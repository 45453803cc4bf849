#!/bin/bash
# Round-2 pass: -m gpu suite, default bench line (resident C2 + host-buffer ABI rates + CPU
# baseline on all cores), C5 strong-scaling rehearsal (2 ranks on 1 GPU) and N=1 strong line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench.log | cut -c1-400 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --scaling strong --total-pairs 2000000 --steps 3 --warmup 1 --rehearse > gpurun_out/strong2.log 2>&1 && echo STRONG2_OK && \
timeout -k 10 300 python bench.py --scaling strong --total-pairs 10000000 --steps 3 --warmup 1 > gpurun_out/strong1.log 2>&1 && echo STRONG1_OK && tail -1 gpurun_out/strong1.log | cut -c1-300
