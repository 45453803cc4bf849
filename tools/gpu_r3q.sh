#!/bin/bash
# Byte-wide H/E planes (BSW_OPT_KERNEL8 = 2) parity + same-box A/B against the int16-plane
# kernel (C2, C3, the QMAX 96 / 64 classes) + a PMC pass of each; busy-device routing of
# coalesced batches (BSW_OPT_BUSY_MIN) in the C++ per-call bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
O=gpurun_out/r3q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_byte_planes.py -x -v --timeout 300 --timeout-method thread > $O/tests_byte.log 2>&1 || { tail -30 $O/tests_byte.log; exit 1; }
tail -1 $O/tests_byte.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "coalesced or small_batch or concurrent or options" > $O/tests_agg.log 2>&1 || { tail -30 $O/tests_agg.log; exit 1; }
tail -1 $O/tests_agg.log
B="--no-cpu --no-host-path --steps 20 --warmup 3"
for rep in 1 2; do
  for k in 1 2; do
    timeout -k 10 200 python bench.py $B --kernel8 $k > $O/c2_k${k}_$rep.json 2>$O/err.log || { tail $O/err.log; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/c2_k${k}_$rep.json').read().strip().splitlines()[-1]);print('C2 k8=$k', d['value'], d['roofline']['launch_ms'])"
  done
done
for k in 1 2; do
  timeout -k 10 200 python bench.py $B --kernel8 $k --cell-bits 8 --h0-hi 130 > $O/c3_k$k.json 2>$O/err.log || { tail $O/err.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c3_k$k.json').read().strip().splitlines()[-1]);print('C3 k8=$k', d['value'], d['roofline']['launch_ms'], d['config']['routing'])"
  for ql in "90 180" "60 120"; do
    set -- $ql
    timeout -k 10 200 python bench.py $B --kernel8 $k --qlen $1 --tlen $2 > $O/q$1_k$k.json 2>$O/err.log || { tail $O/err.log; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/q$1_k$k.json').read().strip().splitlines()[-1]);print('q$1 k8=$k', d['value'], d['roofline']['launch_ms'])"
  done
done
for k in 1 2; do
  OUT=$O/pmc_k$k ARGS="--kernel8 $k --steps 5 --warmup 1 --no-cpu --no-host-path" bash tools/profile.sh > $O/pmc_k$k.log 2>&1 || { echo FAIL pmc $k; tail -5 $O/pmc_k$k.log; exit 1; }
  echo pmc k8=$k done
done
P=bwa-mem2-arm_amd/lib/percall_bench
for bm in 0 8192 4096; do
  for ld in 4 8; do
    timeout -k 10 120 env PERCALL_BUSY_MIN=$bm PERCALL_LEADERS=$ld $P 400000 8 1000 10000 > $O/pc_b${bm}_l$ld.json 2>$O/err.log || { tail $O/err.log; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/pc_b${bm}_l$ld.json'))
print('busy_min=$bm leaders=$ld', [(c['pairs_per_call'], c['coalescing'], c['M_pairs_per_s_1_caller'], c['M_pairs_per_s_8_callers']) for c in d['curve']], d['outputs_identical'])"
  done
done
