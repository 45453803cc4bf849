#!/bin/bash
# host-buffer pipeline change check: parity suites that use host buffers, then the C2 bench line with the ABI rate
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_shim.py tests/test_dist_gpu.py tests/test_batch_file.py tests/test_ext_pipeline.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_hp.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_hp.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_hp.log 2>&1 && python -c "
import json; d=json.loads(open('gpurun_out/bench_hp.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['launch_ms'], d['abi_inclusive_value'], json.dumps(d['abi_inclusive']))"
