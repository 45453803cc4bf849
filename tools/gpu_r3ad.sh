#!/bin/bash
# Coalescing leader linger as an option (BSW_OPT_COALESCE_LINGER, default 30 us): coalescing /
# options / busy-routing tests, C++ per-call bench at the default x2 and with linger 0 x1.
set -o pipefail
O=gpurun_out/r3ad; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread -k "coalesced or options or busy_device or concurrent or small_batch" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P=bwa-mem2-arm_amd/lib/percall_bench
for v in "30 1" "0 1" "30 2"; do
  set -- $v
  timeout -k 10 120 env PERCALL_LINGER=$1 $P 400000 8 1000 4000 10000 16000 > $O/pc_l$1_$2.json 2>$O/err.log || { tail $O/err.log; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/pc_l$1_$2.json'))
print('linger $1 rep $2', [(c['pairs_per_call'], c['latency_ms_median'], c['M_pairs_per_s_8_callers']) for c in d['curve'] if c['coalescing']], d['outputs_identical'])"
done
