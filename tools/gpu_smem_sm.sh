#!/bin/bash
# State-machine SMEM walk: parity (FM-index + chaining tests on the variant library), then the
# phase probe at 1 Gb for the loop form (in-tree) and the state machine.
set -o pipefail
mkdir -p gpurun_out/sm
BSW_HIP_LIB=$PWD/abtmp/libbsw_hip_sm.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_fmi.py tests/test_memchain.py > gpurun_out/sm/tests.log 2>&1 || { tail -30 gpurun_out/sm/tests.log; exit 1; }
tail -1 gpurun_out/sm/tests.log
for v in loop sm; do
  if [ $v = loop ]; then unset BSW_HIP_LIB; else export BSW_HIP_LIB=$PWD/abtmp/libbsw_hip_sm.so; fi
  echo "== $v"; timeout -k 10 300 python -u tools/smem_phase_probe.py 1000 2000000 2>&1 | grep -v generated | grep text | tee gpurun_out/sm/probe_$v.txt
done
