#!/bin/bash
# Same-box A/B on the C3 line (22% of pairs on the int16 lane kernel): in-tree library vs
# lib/libbsw_hip_base.so, alternating, then the -m gpu suite.  Output: gpurun_out/abc3/
set -o pipefail
mkdir -p gpurun_out/abc3
AB="$PWD/bwa-mem2-arm_amd/lib/libbsw_hip_base.so"
for rep in 1 2; do
  for lib in "$AB" ""; do
    BSW_HIP_LIB=$lib timeout -k 10 200 python bench.py --cell-bits 8 --h0-hi 130 --no-cpu --no-host-path > gpurun_out/abc3/ab.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/abc3/ab.log').read().strip().splitlines()[-1]); print('rep=$rep lib=${lib##*/}', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abc3/gpu_tests.log 2>&1 || { tail -30 gpurun_out/abc3/gpu_tests.log; exit 1; }
tail -2 gpurun_out/abc3/gpu_tests.log
