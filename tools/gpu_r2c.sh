#!/bin/bash
# host-path pipeline check: the host-pipeline tests, the bench line, a chunk-size sweep, the
# 2-rank strong rehearsal and the N=1 strong line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_dist_gpu.py -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_c.log 2>&1 && echo TESTS_OK && \
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 && echo BENCH_OK && \
timeout -k 10 300 python tools/host_chunk_sweep.py > gpurun_out/chunk_sweep.log 2>&1 && echo SWEEP_OK && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --scaling strong --total-pairs 2000000 --steps 3 --warmup 1 --rehearse > gpurun_out/strong2.log 2>&1 && echo STRONG2_OK && \
timeout -k 10 300 python bench.py --scaling strong --total-pairs 10000000 --steps 3 --warmup 1 > gpurun_out/strong1.log 2>&1 && echo STRONG1_OK
