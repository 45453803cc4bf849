#!/bin/bash
# Secondary bench lines (GPU box, repo root): C3 routing, C4 extension pipeline, mate rescue.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload mate --steps 5 --warmup 1 > gpurun_out/bench_mate.log 2>&1
tail -1 gpurun_out/bench_mate.log
timeout -k 10 300 python bench.py --cell-bits 8 --h0-hi 105 --no-cpu > gpurun_out/bench_c3.log 2>&1
tail -1 gpurun_out/bench_c3.log
timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1
tail -1 gpurun_out/bench_c4.log
