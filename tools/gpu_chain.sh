#!/bin/bash
# GPU chain2aln: parity tests, then the C4 line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_chain.py tests/test_ext_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_chain.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_chain.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_c4_gpu.log 2>&1 || exit 1
tail -c 1500 gpurun_out/bench_c4_gpu.log
