#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_global.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_o.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python bench.py --workload global --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_global.log 2>&1 && echo GLOBAL_OK && python -c "
import json; d=json.loads(open('gpurun_out/bench_global.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['launch_ms'], d['roofline']['frac'], d['score_only_kernel_ms'])"
tail -2 gpurun_out/gpu_tests_o.log
