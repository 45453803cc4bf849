#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_chain.py tests/test_ext_pipeline.py -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_l.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python bench.py --workload c4 --reads 1000000 --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1 && echo C4_OK && tail -1 gpurun_out/bench_c4.log | cut -c1-1500
tail -5 gpurun_out/gpu_tests_l.log
