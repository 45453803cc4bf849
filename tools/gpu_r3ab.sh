#!/bin/bash
# Row-group kernel with the z-drop gap extensions pinned in registers (no per-row kernarg load):
# group-kernel parity tests, busy-routing parity, C++ per-call bench x2, device-call probe.
set -o pipefail
O=gpurun_out/r3ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "group_kernel or small_batch or busy_device or coalesced" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P=bwa-mem2-arm_amd/lib/percall_bench
for rep in 1 2; do
  timeout -k 10 120 $P 400000 8 1000 4000 10000 16000 > $O/pc_$rep.json 2>$O/err.log || { tail $O/err.log; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/pc_$rep.json'))
print('rep $rep', [(c['pairs_per_call'], c['coalescing'], c['latency_ms_median'], c['M_pairs_per_s_8_callers']) for c in d['curve']], d['outputs_identical'])"
done
timeout -k 10 200 python bench.py --pairs 16000 --no-cpu --no-host-path --steps 50 --warmup 5 > $O/dev16k.log 2>&1 || { tail $O/dev16k.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/dev16k.log').read().strip().splitlines()[-1]);print('device 16K', d['value'], d['roofline']['kernel'], d['roofline']['launch_ms'])"
