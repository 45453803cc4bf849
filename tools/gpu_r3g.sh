#!/bin/bash
# Row-group kernel: parity tests, then the per-call curve with it on / off (C++ callers).
set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  > gpurun_out/r3g/tests.log 2>&1 || { tail -30 gpurun_out/r3g/tests.log; exit 1; }
tail -3 gpurun_out/r3g/tests.log
for G in 1 0; do
  PERCALL_GROUP=$G timeout -k 10 150 ./bwa-mem2-arm_amd/lib/percall_bench 1000000 8 1000 4000 10000 16000 > gpurun_out/r3g/percall_G$G.json 2>&1 || { cat gpurun_out/r3g/percall_G$G.json; exit 1; }
  echo "G=$G"; cat gpurun_out/r3g/percall_G$G.json
done
