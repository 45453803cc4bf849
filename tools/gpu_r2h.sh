#!/bin/bash
# kernel A/B: parity tests of the DP kernels, then the bench line (no host path / CPU legs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_batch_file.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_h.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python bench.py --no-cpu --no-host-path --steps 20 --warmup 3 > gpurun_out/bench_h.log 2>&1 && echo BENCH_OK && python -c "
import json; d=json.loads(open('gpurun_out/bench_h.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['launch_ms'], d['roofline']['frac'])"
