#!/bin/bash
# Coalescing leader linger A/B (BSW_AGG_LINGER_US 0 = off / 30 / 80): a leader that starts while
# another batch is in flight waits that long for the just-returned callers' next calls.
set -o pipefail
O=gpurun_out/r3ac; mkdir -p $O
P=bwa-mem2-arm_amd/lib/percall_bench
for rep in 1 2; do
  for lg in 0 30 80; do
    timeout -k 10 120 env BSW_AGG_LINGER_US=$lg $P 400000 8 1000 4000 10000 16000 > $O/pc_l${lg}_$rep.json 2>$O/err.log || { tail $O/err.log; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/pc_l${lg}_$rep.json'))
print('linger $lg rep $rep', [(c['pairs_per_call'], c['latency_ms_median'], c['M_pairs_per_s_8_callers']) for c in d['curve'] if c['coalescing']], d['outputs_identical'])"
  done
done
