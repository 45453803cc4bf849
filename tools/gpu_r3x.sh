#!/bin/bash
# Round-3 refresh of the current tree: the whole GPU suite, smoke(), the default bench line,
# and a small-batch routing sweep (BSW_OPT_SMALL_BATCH 16384 default vs 32768: 16K-32K coalesced
# batches on the 16-lane row-group kernel instead of its quad form), C++ per-call bench x2.
set -o pipefail
O=gpurun_out/r3x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
P=bwa-mem2-arm_amd/lib/percall_bench
for rep in 1 2; do
  for sb in 16384 32768; do
    timeout -k 10 120 env PERCALL_SMALL=$sb $P 400000 8 1000 10000 16000 > $O/pc_s${sb}_$rep.json 2>$O/err.log || { tail $O/err.log; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/pc_s${sb}_$rep.json'))
print('small_batch=$sb rep $rep', [(c['pairs_per_call'], c['coalescing'], c['M_pairs_per_s_1_caller'], c['M_pairs_per_s_8_callers']) for c in d['curve']], d['outputs_identical'])"
  done
done
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -c 2500 $O/bench.log; echo
