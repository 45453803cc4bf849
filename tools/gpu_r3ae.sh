#!/bin/bash
# Linger A/B with more repetitions: BSW_OPT_COALESCE_LINGER 0 vs 30 us, interleaved x5, 1K / 10K pairs per call, 8 callers.
set -o pipefail
O=gpurun_out/r3ae; mkdir -p $O
P=bwa-mem2-arm_amd/lib/percall_bench
for rep in 1 2 3 4 5; do
  line="rep $rep"
  for lg in 0 30; do
    timeout -k 10 120 env PERCALL_LINGER=$lg $P 400000 8 1000 10000 > $O/pc_l${lg}_$rep.json 2>$O/err.log || { tail $O/err.log; exit 1; }
    line="$line | linger $lg: $(python3 -c "
import json;d=json.load(open('$O/pc_l${lg}_$rep.json'))
print(' '.join('%d:%.1f' % (c['pairs_per_call'], c['M_pairs_per_s_8_callers']) for c in d['curve'] if c['coalescing']), d['outputs_identical'])")"
  done
  echo "$line"
done
