#!/bin/bash
# SMEM seeding: parity tests, then the bench at 16 Mb (index inside the 256 MB MALL) and 256 Mb (not)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fmi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_fmi.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_fmi.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload smem --steps 3 --warmup 1 > gpurun_out/bench_smem16.log 2>&1 || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/bench_smem16.log').read().strip().splitlines()[-1]); print('16Mb', d['value'], d['roofline']['launch_ms'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'), d['outputs_identical_to_oracle_sample'])"
timeout -k 10 600 python bench.py --workload smem --smem-ref-mb 256 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_smem256.log 2>&1 || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/bench_smem256.log').read().strip().splitlines()[-1]); print('256Mb', d['value'], d['roofline']['launch_ms'], d['roofline']['frac'], d['config']['index_build_s'], d['config']['index_device_bytes'])"
