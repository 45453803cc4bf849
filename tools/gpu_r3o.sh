#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3o
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/r3o/tests.log 2>&1 || { tail -30 gpurun_out/r3o/tests.log; exit 1; }
tail -1 gpurun_out/r3o/tests.log
timeout -k 10 200 python -u tools/mid_batch_probe.py 2>&1 | tee gpurun_out/r3o/mid.txt
timeout -k 10 150 ./bwa-mem2-arm_amd/lib/percall_bench 1000000 8 1000 4000 10000 16000 > gpurun_out/r3o/percall.json 2>&1 || { cat gpurun_out/r3o/percall.json; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r3o/percall.json'))
print(' '.join('%d%s:%.3fms/%.1f/%.1f' % (c['pairs_per_call'], 'c' if c['coalescing'] else 'n', c['latency_ms_median'], c['M_pairs_per_s_1_caller'], c['M_pairs_per_s_8_callers']) for c in d['curve']), d['outputs_identical'])"
