#!/bin/bash
# SMEM workgroup size A/B: 64 (in-tree) / 256 / 512 threads per workgroup, phase probe at 1 Gb.
set -o pipefail
mkdir -p gpurun_out/probe
for v in b64 b256 b512; do
  if [ $v = b64 ]; then unset BSW_HIP_LIB; else export BSW_HIP_LIB=$PWD/abtmp/libbsw_hip_$v.so; fi
  echo "== $v"; timeout -k 10 300 python -u tools/smem_phase_probe.py 1000 2000000 2>&1 | grep -v generated | grep text | tee gpurun_out/probe/block_$v.txt
done
