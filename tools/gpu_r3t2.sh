#!/bin/bash
# Kernel trace of the C++ per-call bench at 1K pairs x 8 callers (coalescing on): queue ids and
# overlap of the coalesced batches' row-group launches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
rm -rf gpurun_out/t1k
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/t1k -- bwa-mem2-arm_amd/lib/percall_bench 200000 8 1000 > gpurun_out/t1k.log 2>&1 || { tail gpurun_out/t1k.log; exit 1; }
grep '^{' gpurun_out/t1k.log | cut -c1-400
