#!/bin/bash
# Full round refresh on the GPU box: every GPU test, the default bench line, rocprofv3 passes,
# and the secondary bench lines (C3 routing, C4 pipeline, mate rescue, global + CIGAR).
set -euo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log | cut -c1-200
OUT=gpurun_out/prof bash tools/profile.sh
bash tools/gpu_benches.sh | cut -c1-160
timeout -k 10 300 python bench.py --workload global --steps 5 --warmup 1 > gpurun_out/bench_global.log 2>&1
tail -1 gpurun_out/bench_global.log | cut -c1-160
echo all-done
