#!/bin/bash
# Coalescing policy sweep: small-batch threshold x leaders, C++ callers.
set -o pipefail
mkdir -p gpurun_out/r3k
for SB in 16384 32768; do for L in 2 4 8; do
  PERCALL_SMALL=$SB PERCALL_LEADERS=$L timeout -k 10 120 ./bwa-mem2-arm_amd/lib/percall_bench 1000000 8 1000 4000 10000 > gpurun_out/r3k/p_${SB}_$L.json 2>&1 || { cat gpurun_out/r3k/p_${SB}_$L.json; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r3k/p_${SB}_$L.json'))
print('SB=$SB L=$L', ' '.join('%d%s:%.1f/%.1f' % (c['pairs_per_call'], 'c' if c['coalescing'] else 'n', c['M_pairs_per_s_1_caller'], c['M_pairs_per_s_8_callers']) for c in d['curve']))"
done; done
