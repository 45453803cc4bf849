#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_ext_pipeline.py tests/test_dist_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_d.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python tools/host_chunk_sweep.py > gpurun_out/chunk_sweep.log 2>&1 && echo SWEEP_OK && cat gpurun_out/chunk_sweep.log && \
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench.log | cut -c1-250
