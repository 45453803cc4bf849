#!/bin/bash
# (1) host pipeline A/B (tools/gpu_r3u.sh); (2) the pipeline's invalid-pair test; (3) SMEM walk
# occupancy A/B at C4 scale (wide index, 3 Gb): product build vs BSW_SMEM_WAVES 5 / 6 / 8 builds.
set -o pipefail
O=gpurun_out/r3v; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dist_gpu.py -x -q --timeout 240 --timeout-method thread -k "invalid_pair or host_pipeline or rccl" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
bash tools/gpu_r3u.sh || exit 1
L=$PWD/bwa-mem2-arm_amd/lib
for v in base w5 w6 w8 base; do
  if [ $v = base ]; then unset BSW_HIP_LIB; else export BSW_HIP_LIB=$L/libbsw_hip_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload c4mem --reads 2000000 --ref-mb 3000 --steps 3 --warmup 1 > $O/c4_$v.log 2>&1 || { tail -20 $O/c4_$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c4_$v.log').read().strip().splitlines()[-1]);print('$v', d['reads_per_s_M'], d['stage_ms'], d['smem_kernel_ms'])"
done
unset BSW_HIP_LIB
