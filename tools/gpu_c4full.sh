#!/bin/bash
# C4 at BASELINE scale through the GPU front end: 10M PE 150 bp reads vs a 3 Gb random reference,
# wide (64-bit) GPU-built FM-index, SMEM seeding -> chaining -> mem_chain2aln, all resident.
set -o pipefail
mkdir -p gpurun_out/c4full
timeout -k 10 1000 python -u bench.py --workload c4mem --reads 10000000 --ref-mb 3000 --steps 3 --warmup 1 > gpurun_out/c4full/bench_c4mem_3gb.log 2>&1 || { tail -30 gpurun_out/c4full/bench_c4mem_3gb.log; exit 1; }
tail -c 3000 gpurun_out/c4full/bench_c4mem_3gb.log
