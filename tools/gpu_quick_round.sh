#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
OUT=gpurun_out/prof bash tools/profile.sh
