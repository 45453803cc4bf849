#!/bin/bash
# Coalescing threshold A/B (BSW_OPT_COALESCE 32768 = round-3 default vs 2048), interleaved x3,
# C++ per-call bench, 8 callers, 1K / 4K / 10K / 16K pairs per call.
set -o pipefail
O=gpurun_out/r3s2; mkdir -p $O
P=bwa-mem2-arm_amd/lib/percall_bench
for rep in 1 2 3; do
  for co in 32768 2048; do
    timeout -k 10 120 env PERCALL_COALESCE=$co $P 400000 8 1000 4000 10000 16000 > $O/pc_c${co}_$rep.json 2>$O/err.log || { tail $O/err.log; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/pc_c${co}_$rep.json'))
print('coalesce=$co rep $rep', [(c['pairs_per_call'], c['coalescing'], c['M_pairs_per_s_1_caller'], c['M_pairs_per_s_8_callers']) for c in d['curve']], d['outputs_identical'])"
  done
done
