#!/bin/bash
# GPU test pass (gpurun): the whole -m gpu suite, one process, per-test timeout; log under gpurun_out/.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/gpu_tests.log 2>&1
tail -3 gpurun_out/gpu_tests.log
