#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 1 > gpurun_out/bench_c4.log 2>&1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c4.log').read().strip().splitlines()[-1]);print('c4', d['value'], d['reads_per_s_M'], d['dp_kernel_ms_per_step'], d['ms_per_step'], d['pcie_inclusive_reads_per_s_M'], d['device_host_paths_identical'])"
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_c2.log 2>&1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c2.log').read().strip().splitlines()[-1]);print('c2', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
