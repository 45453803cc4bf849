#!/bin/bash
# Round-2 final refresh, part C (after the wave-kernel change): long-read lines, C1, small-batch table
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 300 python bench.py --qlen 250 --tlen 350 --pairs 500000 --no-cpu --no-host-path > gpurun_out/r02/bench_long250.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --qlen 500 --tlen 600 --pairs 200000 --no-cpu --no-host-path > gpurun_out/r02/bench_long500.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --qlen 1000 --tlen 1100 --pairs 100000 --no-cpu --no-host-path > gpurun_out/r02/bench_long1000.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c1 --steps 5 --warmup 1 > gpurun_out/r02/bench_c1.log 2>&1 || exit 1
timeout -k 10 240 python3 tools/small_batch_latency.py > gpurun_out/r02/small_batch_latency.txt 2>&1 || exit 1
for f in gpurun_out/r02/bench_long*.log gpurun_out/r02/bench_c1.log; do echo "$f $(tail -1 $f | cut -c1-120)"; done
cat gpurun_out/r02/small_batch_latency.txt
echo final-c-done
