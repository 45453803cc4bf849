#!/bin/bash
# C3 study: occupancy microbenchmark + routing/fallback runs + the C3 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 5 120 ./tools/pc_branch_bench > gpurun_out/pc_branch_bench.log 2>&1 && echo MB_OK && \
timeout -k 10 400 python tools/c3_study.py > gpurun_out/c3_study.json 2> gpurun_out/c3_study.log && echo C3_OK && \
timeout -k 10 300 python bench.py --cell-bits 8 --h0-hi 130 --no-host-path > gpurun_out/bench_c3.log 2>&1 && echo BENCH_C3_OK
