#!/bin/bash
# C4 at BASELINE scale: 10M PE reads vs a 3 Gb reference (chains, mem_chain2aln) -- one bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --workload c4 --reads 10000000 --ref-mb 3000 --steps 2 --warmup 1 > gpurun_out/bench_c4_full_pe.log 2>&1; rc=$?
tail -c 2500 gpurun_out/bench_c4_full_pe.log
exit $rc
