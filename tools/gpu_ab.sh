#!/bin/bash
# A/B of the product library against the experiment build lib/libbsw_hip_ab.so (make ab AB_FLAGS=...)
# on one box, alternating, C2 shape and (optionally) a short class: prints value / kernel ms per run
set -o pipefail
mkdir -p gpurun_out
AB="$PWD/bwa-mem2-arm_amd/lib/libbsw_hip_ab.so"
for rep in 1 2; do
  for lib in "" "$AB"; do
    for q in ${AB_QLENS:-150}; do
      BSW_HIP_LIB=$lib timeout -k 10 200 python bench.py --qlen $q --tlen $((2*q)) --no-cpu --no-host-path > gpurun_out/ab.log 2>&1 || exit 1
      python -c "
import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('rep=$rep lib=${lib##*/} qlen=$q', d['value'], d['roofline']['launch_ms'])"
    done
  done
done
