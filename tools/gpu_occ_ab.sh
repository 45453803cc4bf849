#!/bin/bash
# occupancy A/B on the packed-column kernel: QMAX=96 class (170 VGPRs -> 3 waves/SIMD) vs the same
# kernel capped at 2 waves/SIMD by 11 KB of dynamic LDS per one-wave workgroup (8 per CU)
set -o pipefail
for lib in "" "$PWD/bwa-mem2-arm_amd/lib/libbsw_hip_pad.so"; do
  for q in 90 60; do
    BSW_HIP_LIB=$lib timeout -k 10 200 python bench.py --qlen $q --tlen $((2*q)) --no-cpu --no-host-path > gpurun_out/occ.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/occ.log').read().strip().splitlines()[-1]); print('lib=${lib##*/} qlen=$q', d['value'], d['roofline']['kernel'], d['roofline']['launch_ms'])"
  done
done
