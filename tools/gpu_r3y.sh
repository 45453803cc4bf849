#!/bin/bash
# Small-batch default 32768 (16-lane row-group form up to 32K): routing / parity tests, C++ per-call x2.
set -o pipefail
O=gpurun_out/r3y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "small_batch or group_kernel or coalesced or concurrent" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P=bwa-mem2-arm_amd/lib/percall_bench
for rep in 1 2; do
  timeout -k 10 120 $P 400000 8 1000 4000 10000 16000 24000 > $O/pc_$rep.json 2>$O/err.log || { tail $O/err.log; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/pc_$rep.json'))
print('rep $rep', [(c['pairs_per_call'], c['coalescing'], c['latency_ms_median'], c['M_pairs_per_s_1_caller'], c['M_pairs_per_s_8_callers']) for c in d['curve']], d['outputs_identical'])"
done
