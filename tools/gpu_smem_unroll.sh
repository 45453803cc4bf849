#!/bin/bash
# SMEM backward-sweep unroll A/B (1 / 2 (in-tree) / 4) with the phase probe, then parity.
set -o pipefail
mkdir -p gpurun_out/probe
for v in u1 u2 u4; do
  if [ $v = u2 ]; then unset BSW_HIP_LIB; else export BSW_HIP_LIB=$PWD/abtmp/libbsw_hip_$v.so; fi
  echo "== $v"; timeout -k 10 300 python -u tools/smem_phase_probe.py 1000 2000000 2>&1 | grep -v generated | grep text | tee gpurun_out/probe/unroll_$v.txt
done
unset BSW_HIP_LIB
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fmi.py tests/test_memchain.py 2>&1 | tail -1
