#!/bin/bash
# Round-2 final refresh, part B: secondary bench lines (mate, global, C3, C4 seeds, C1, SMEM,
# C4 PE 1M/64 Mb, long reads).  Output: gpurun_out/r02/
set -o pipefail
mkdir -p gpurun_out/r02
for w in mate global; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 > gpurun_out/r02/bench_$w.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --cell-bits 8 --h0-hi 130 --no-cpu --no-host-path > gpurun_out/r02/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c4seed --steps 3 --warmup 1 > gpurun_out/r02/bench_c4seed.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c1 --steps 5 --warmup 1 > gpurun_out/r02/bench_c1.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload smem --steps 3 --warmup 1 > gpurun_out/r02/bench_smem.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/r02/bench_c4_pe.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --qlen 250 --tlen 350 --pairs 500000 --no-cpu --no-host-path > gpurun_out/r02/bench_long250.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --qlen 500 --tlen 600 --pairs 200000 --no-cpu --no-host-path > gpurun_out/r02/bench_long500.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --qlen 1000 --tlen 1100 --pairs 100000 --no-cpu --no-host-path > gpurun_out/r02/bench_long1000.log 2>&1 || exit 1
for f in gpurun_out/r02/bench*.log; do echo "$f $(tail -1 $f | cut -c1-150)"; done
echo final-b-done
