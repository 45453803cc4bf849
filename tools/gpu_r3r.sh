#!/bin/bash
# Coalescing policy sweep in the C++ per-call bench: leaders 1 / 2 / 4 x busy-device routing
# (BSW_OPT_BUSY_MIN 0 = off, 8192), 1K and 10K pairs per call, 8 callers; default repeated.
set -o pipefail
O=gpurun_out/r3r; mkdir -p $O
P=bwa-mem2-arm_amd/lib/percall_bench
for cfg in "8192 4" "8192 4" "0 1" "8192 1" "0 2" "8192 2" "16384 2" "8192 3"; do
  set -- $cfg
  timeout -k 10 120 env PERCALL_BUSY_MIN=$1 PERCALL_LEADERS=$2 $P 400000 8 1000 10000 > $O/pc_b$1_l$2.json 2>$O/err.log || { tail $O/err.log; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/pc_b$1_l$2.json'))
print('busy_min=$1 leaders=$2', [(c['pairs_per_call'], c['coalescing'], c['M_pairs_per_s_1_caller'], c['M_pairs_per_s_8_callers']) for c in d['curve']], d['outputs_identical'])"
done
