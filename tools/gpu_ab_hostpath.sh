#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/abh
timeout -k 10 300 python tools/ab_hostpath.py bwa-mem2-arm_amd/lib/libbsw_hip_base.so bwa-mem2-arm_amd/lib/libbsw_hip.so 25 2>&1 | tee gpurun_out/abh/interleaved.txt
