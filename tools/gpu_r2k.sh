#!/bin/bash
# long-read shapes on the wave kernel (vs the wide kernel), resident batches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --qlen 250 --tlen 350 --pairs 500000 --steps 5 --warmup 1 --no-host-path > gpurun_out/bench_long250.log 2>&1 && echo L250_OK && \
timeout -k 10 300 python bench.py --qlen 500 --tlen 600 --pairs 200000 --steps 5 --warmup 1 --no-host-path --no-cpu > gpurun_out/bench_long500.log 2>&1 && echo L500_OK && \
timeout -k 10 300 python bench.py --qlen 1000 --tlen 1100 --pairs 100000 --steps 5 --warmup 1 --no-host-path --no-cpu > gpurun_out/bench_long1000.log 2>&1 && echo L1000_OK
for f in gpurun_out/bench_long*.log; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['roofline']['kernel'], d['roofline']['launch_ms'], d['roofline']['frac'], d.get('wide_kernel_comparison'), (d.get('cpu_baseline') or {}).get('value'))"; done
