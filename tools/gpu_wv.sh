#!/bin/bash
# wave-kernel change check: parity suite (golden sets and random batches through the wave kernel,
# small-batch routing), long-read bench line, small-batch latency table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_wv.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_wv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --qlen 250 --tlen 350 --pairs 500000 --no-cpu --no-host-path > gpurun_out/bench_wv250.log 2>&1 || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/bench_wv250.log').read().strip().splitlines()[-1]); print('long250', d['value'], d['roofline']['launch_ms'], d['roofline']['frac'])"
timeout -k 10 240 python3 tools/small_batch_latency.py | head -6
