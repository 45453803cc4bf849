#!/bin/bash
# Round 3: the seeding -> chaining -> extension front end on the GPU (tests/test_memchain.py),
# then its bench lines (C1 on the reference's own data, C4 front end at 64 Mb).
set -o pipefail
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest tests/test_memchain.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3b/memchain.log 2>&1 || { tail -40 gpurun_out/r3b/memchain.log; exit 1; }
tail -8 gpurun_out/r3b/memchain.log
timeout -k 10 300 python bench.py --workload c1 --steps 10 --warmup 2 > gpurun_out/r3b/bench_c1.log 2>&1 || { tail -30 gpurun_out/r3b/bench_c1.log; exit 1; }
tail -c 2500 gpurun_out/r3b/bench_c1.log; echo
timeout -k 10 400 python bench.py --workload c4mem --reads 1000000 --ref-mb 64 --steps 5 --warmup 1 > gpurun_out/r3b/bench_c4mem.log 2>&1 || { tail -30 gpurun_out/r3b/bench_c4mem.log; exit 1; }
tail -c 2500 gpurun_out/r3b/bench_c4mem.log; echo
