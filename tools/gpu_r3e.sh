#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_dist.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3e/dist.log 2>&1 || { tail -40 gpurun_out/r3e/dist.log; exit 1; }
tail -6 gpurun_out/r3e/dist.log
