#!/bin/bash
# pc kernel change check: parity suite for the extension kernels, then the C2 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_shim.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_pc.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_pc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-host-path > gpurun_out/bench_pc.log 2>&1 && python -c "
import json; d=json.loads(open('gpurun_out/bench_pc.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['launch_ms'], d['roofline']['frac'])"
