#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_j.log 2>&1 && echo TESTS_OK
tail -30 gpurun_out/gpu_tests_j.log | cut -c1-300
