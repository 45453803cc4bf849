#!/bin/bash
# Device extension pipeline on the GPU box: parity tests + C4 bench line.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ext_pipeline.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_ext_tests.log 2>&1
tail -3 gpurun_out/gpu_ext_tests.log
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 1 > gpurun_out/bench_c4.log 2>&1
tail -1 gpurun_out/bench_c4.log
