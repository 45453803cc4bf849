#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3d
for L in 2 4 8; do
  PERCALL_LEADERS=$L timeout -k 10 120 ./bwa-mem2-arm_amd/lib/percall_bench 1000000 8 1000 10000 > gpurun_out/r3d/percall_L$L.json 2>&1 || { cat gpurun_out/r3d/percall_L$L.json; exit 1; }
  echo "L=$L"; cat gpurun_out/r3d/percall_L$L.json
done
BSW_DEBUG_AGG=1 PERCALL_LEADERS=4 timeout -k 10 120 ./bwa-mem2-arm_amd/lib/percall_bench 1000000 8 1000 10000 > gpurun_out/r3d/debug.log 2>&1 || { tail -5 gpurun_out/r3d/debug.log; exit 1; }
grep "agg batch" gpurun_out/r3d/debug.log | awk 'NR%150==0' | head -40
