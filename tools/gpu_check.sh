#!/bin/bash
# Quick GPU check: full -m gpu suite + the default C2 bench line. Output: gpurun_out/chk/
set -o pipefail
mkdir -p gpurun_out/chk
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/gpu_tests.log 2>&1 || { tail -30 gpurun_out/chk/gpu_tests.log; exit 1; }
tail -2 gpurun_out/chk/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/chk/bench.log 2>&1 || { tail -30 gpurun_out/chk/bench.log; exit 1; }
tail -c 1500 gpurun_out/chk/bench.log; echo
