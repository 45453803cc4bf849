#!/bin/bash
# Where a small call's time goes: per-batch host timeline (BSW_DEBUG_AGG) + kernel trace.
set -o pipefail
mkdir -p gpurun_out/r3h
export TMPDIR=/tmp
BSW_DEBUG_AGG=1 timeout -k 10 120 ./bwa-mem2-arm_amd/lib/percall_bench 200000 8 1000 10000 > gpurun_out/r3h/debug.json 2> gpurun_out/r3h/debug.log || { tail -5 gpurun_out/r3h/debug.log; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3h/prof -o run -- ./bwa-mem2-arm_amd/lib/percall_bench 200000 8 1000 10000 > gpurun_out/r3h/prof.log 2>&1 || { tail -5 gpurun_out/r3h/prof.log; exit 1; }
find gpurun_out/r3h/prof -name "*stats*" | head
