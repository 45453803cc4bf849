#!/bin/bash
# timeline of the C2 device step (kernels + copies) for the per-step overhead outside the DP kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf gpurun_out/c2t
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/c2t -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-host-path > gpurun_out/c2t.log 2>&1
