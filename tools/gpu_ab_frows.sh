#!/bin/bash
# Same-box A/B on the global (ksw_global2 + CIGAR) and mate-rescue lines: in-tree library vs
# lib/libbsw_hip_base.so, alternating, then the -m gpu suite.  Output: gpurun_out/abf/
set -o pipefail
mkdir -p gpurun_out/abf
AB="$PWD/bwa-mem2-arm_amd/lib/libbsw_hip_base.so"
for rep in 1 2; do
  for wl in global mate; do
    for lib in "$AB" ""; do
      BSW_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload $wl --steps 5 --warmup 1 --no-cpu > gpurun_out/abf/ab.log 2>&1 || exit 1
      python -c "
import json; d=json.loads(open('gpurun_out/abf/ab.log').read().strip().splitlines()[-1]); print('rep=$rep $wl lib=${lib##*/}', d['value'], d['ms_per_step'])"
    done
  done
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abf/gpu_tests.log 2>&1 || { tail -30 gpurun_out/abf/gpu_tests.log; exit 1; }
tail -2 gpurun_out/abf/gpu_tests.log
