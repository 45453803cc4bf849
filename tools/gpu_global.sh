#!/bin/bash
# Global-alignment row on the GPU box: parity tests, bench line, kernel trace.
set -euo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests/test_global.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_global_tests.log 2>&1
tail -3 gpurun_out/gpu_global_tests.log
timeout -k 10 300 python bench.py --workload global --steps 5 --warmup 1 > gpurun_out/bench_global.log 2>&1
tail -1 gpurun_out/bench_global.log
rm -rf gpurun_out/prof_global
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_global -- python3 bench.py --workload global --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_global.log 2>&1
echo global-done
