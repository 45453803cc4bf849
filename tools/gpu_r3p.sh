#!/bin/bash
# Re-entry check of the rebuilt tree: GPU suite, default bench line, and the coalesced
# small-call path's per-batch breakdown (BSW_DEBUG_AGG) at 1K and 10K pairs x 8 callers.
set -o pipefail
mkdir -p gpurun_out/r3p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3p/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3p/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3p/gpu_tests.log
timeout -k 10 120 env BSW_DEBUG_AGG=1 bwa-mem2-arm_amd/lib/percall_bench 400000 8 1000 > gpurun_out/r3p/pc1k.json 2> gpurun_out/r3p/pc1k.err || exit 1
timeout -k 10 120 env BSW_DEBUG_AGG=1 bwa-mem2-arm_amd/lib/percall_bench 400000 8 10000 > gpurun_out/r3p/pc10k.json 2> gpurun_out/r3p/pc10k.err || exit 1
cat gpurun_out/r3p/pc1k.json gpurun_out/r3p/pc10k.json
timeout -k 10 400 python bench.py > gpurun_out/r3p/bench.log 2>&1 || { tail -30 gpurun_out/r3p/bench.log; exit 1; }
tail -c 3000 gpurun_out/r3p/bench.log; echo
