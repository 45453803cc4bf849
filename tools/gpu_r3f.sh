#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3f
timeout -k 10 700 python -u -m pytest tests/test_fmi.py tests/test_memchain.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r3f/fmi.log 2>&1 || { tail -40 gpurun_out/r3f/fmi.log; exit 1; }
tail -5 gpurun_out/r3f/fmi.log
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_dist.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3f/dist.log 2>&1 || { tail -40 gpurun_out/r3f/dist.log; exit 1; }
tail -5 gpurun_out/r3f/dist.log
