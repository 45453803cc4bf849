#!/bin/bash
# Coalesced small batches staged on the leader thread (< 4 MB of bases) vs through the shared host
# pool (the previous build, lib/percall_bench_prev -> libbsw_hip_prev.so): C++ per-call bench,
# 8 callers, interleaved x3.
set -o pipefail
O=gpurun_out/r3z; mkdir -p $O
L=bwa-mem2-arm_amd/lib
for rep in 1 2 3; do
  for v in new prev; do
    P=$L/percall_bench; [ $v = prev ] && P=$L/percall_bench_prev
    timeout -k 10 120 $P 400000 8 1000 4000 10000 > $O/pc_${v}_$rep.json 2>$O/err.log || { tail $O/err.log; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/pc_${v}_$rep.json'))
print('$v rep $rep', [(c['pairs_per_call'], c['M_pairs_per_s_1_caller'], c['M_pairs_per_s_8_callers']) for c in d['curve'] if c['coalescing']], d['outputs_identical'])"
  done
done
