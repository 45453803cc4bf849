#!/bin/bash
# Same-box A/B of the in-tree library against lib/libbsw_hip_base.so (tools/ab_lib.sh), then the
# whole -m gpu suite on the in-tree library.  Output: gpurun_out/absuite/
set -o pipefail
mkdir -p gpurun_out/absuite
bash tools/ab_lib.sh > gpurun_out/absuite/ab.txt 2>&1 || { cat gpurun_out/absuite/ab.txt; exit 1; }
cat gpurun_out/absuite/ab.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/absuite/gpu_tests.log 2>&1 || { tail -30 gpurun_out/absuite/gpu_tests.log; exit 1; }
tail -2 gpurun_out/absuite/gpu_tests.log
