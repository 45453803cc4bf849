#!/bin/bash
# Secondary bench lines that run on the packed-column kernel (C3, C4 PE chains, C4 seeds, C1),
# refreshed after a pc_kernel change.  Output: gpurun_out/r02/
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 300 python bench.py --cell-bits 8 --h0-hi 130 --no-cpu --no-host-path > gpurun_out/r02/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/r02/bench_c4_pe.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c4seed --steps 3 --warmup 1 > gpurun_out/r02/bench_c4seed.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c1 --steps 5 --warmup 1 > gpurun_out/r02/bench_c1.log 2>&1 || exit 1
for f in gpurun_out/r02/bench_c3.log gpurun_out/r02/bench_c4_pe.log gpurun_out/r02/bench_c4seed.log gpurun_out/r02/bench_c1.log; do echo "$f $(tail -1 $f | cut -c1-160)"; done
echo pc-lines-done
