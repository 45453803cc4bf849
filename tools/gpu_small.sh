#!/bin/bash
# small-batch routing check: parity suite (kernel classes pinned + small-batch tests), smoke, latency table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_shim.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_small.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 240 python3 tools/small_batch_latency.py
