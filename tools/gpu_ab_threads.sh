#!/bin/bash
# Host pool size A/B (cgroup quota 16 on the box): 16 lanes vs 12 / 8, interleaved in one process.
set -o pipefail
mkdir -p gpurun_out/abt
cp bwa-mem2-arm_amd/lib/libbsw_hip.so /tmp/libbsw_hip_b.so
for T in 16; do
timeout -k 10 300 python tools/ab_hostpath.py bwa-mem2-arm_amd/lib/libbsw_hip.so /tmp/libbsw_hip_b.so 20 16 $T 2>&1 | tee gpurun_out/abt/threads_16_$T.txt
done
