#!/bin/bash
# Round 3 check: this round's new tests first, then the full -m gpu suite and the default C2
# bench line.  Output: gpurun_out/r3a/
set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 600 python -u -m pytest tests/test_chain.py tests/test_ext_pipeline.py tests/test_shim.py tests/test_dist.py \
  "tests/test_gpu_parity.py::test_multi_device_policy_rehearsal" "tests/test_gpu_parity.py::test_extreme_gap_penalties" \
  "tests/test_gpu_parity.py::test_host_pipeline_2bit_pieces_over_8mb" \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3a/new_tests.log 2>&1 || { tail -40 gpurun_out/r3a/new_tests.log; exit 1; }
tail -3 gpurun_out/r3a/new_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3a/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3a/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3a/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r3a/bench.log 2>&1 || { tail -30 gpurun_out/r3a/bench.log; exit 1; }
tail -c 1500 gpurun_out/r3a/bench.log; echo
