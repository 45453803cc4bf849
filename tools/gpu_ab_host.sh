#!/bin/bash
# Same-box A/B of the host-buffer (drop-in) path: in-tree library vs lib/libbsw_hip_base.so,
# alternating; prints the resident value and abi_inclusive_value per run.
set -o pipefail
mkdir -p gpurun_out/abh
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pipeline or host or small or group or coalesc" > gpurun_out/abh/tests.log 2>&1 || { tail -20 gpurun_out/abh/tests.log; exit 1; }
tail -1 gpurun_out/abh/tests.log
for k in 1 2 3; do
for v in base new; do
  if [ $v = base ]; then export BSW_HIP_LIB=$PWD/bwa-mem2-arm_amd/lib/libbsw_hip_base.so; else unset BSW_HIP_LIB; fi
  timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/abh/ab_$v.log 2>&1 || { tail -5 gpurun_out/abh/ab_$v.log; exit 1; }
  echo "$k $v $(python3 -c "import json;d=json.loads(open('gpurun_out/abh/ab_$v.log').read().strip().splitlines()[-1]);print(d['value'], d.get('abi_inclusive_value'), d.get('abi_inclusive',{}).get('fraction_of_resident'))")"
done
done
