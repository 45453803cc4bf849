#!/bin/bash
# C4 lines: 1M PE reads vs 64 Mb, and BASELINE scale (10M PE reads vs 3 Gb)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/bench_c4_pe.log 2>&1 || exit 1
tail -c 1200 gpurun_out/bench_c4_pe.log; echo
timeout -k 10 900 python bench.py --workload c4 --reads 10000000 --ref-mb 3000 --steps 2 --warmup 1 > gpurun_out/bench_c4_full_pe.log 2>&1 || exit 1
tail -c 1500 gpurun_out/bench_c4_full_pe.log
