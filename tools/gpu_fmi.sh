#!/bin/bash
# FM-index seeding row: GPU parity tests, then a short smem bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fmi.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_fmi.log 2>&1; rc=$?
tail -12 gpurun_out/gpu_tests_fmi.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload smem --reads 1000000 --steps 3 --warmup 1 > gpurun_out/bench_smem.log 2>&1; rc=$?
tail -c 3000 gpurun_out/bench_smem.log
exit $rc
