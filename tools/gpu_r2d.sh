#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/h2d_bench > gpurun_out/h2d_bench.log 2>&1 && echo H2D_OK && cat gpurun_out/h2d_bench.log && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_batch_file.py tests/test_dist_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_d.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python tools/host_chunk_sweep.py > gpurun_out/chunk_sweep.log 2>&1 && echo SWEEP_OK && cat gpurun_out/chunk_sweep.log
