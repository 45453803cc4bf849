#!/bin/bash
# Round 3 check: the chain-window / validation tests first, then the full -m gpu suite and the
# default C2 bench line.  Output: gpurun_out/r3a/
set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 600 python -u -m pytest tests/test_chain.py tests/test_ext_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3a/chain_tests.log 2>&1 || { tail -40 gpurun_out/r3a/chain_tests.log; exit 1; }
tail -3 gpurun_out/r3a/chain_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3a/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3a/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3a/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r3a/bench.log 2>&1 || { tail -30 gpurun_out/r3a/bench.log; exit 1; }
tail -c 1500 gpurun_out/r3a/bench.log; echo
