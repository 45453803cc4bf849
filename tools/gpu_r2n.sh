#!/bin/bash
# f-row kernels: global (+CIGAR) and mate rescue -- tests, bench lines, PMC traffic passes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 500 python -u -m pytest tests/test_global.py tests/test_mate_rescue.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_n.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python bench.py --workload global --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_global.log 2>&1 && echo GLOBAL_OK && \
timeout -k 10 300 python bench.py --workload mate --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_mate.log 2>&1 && echo MATE_OK && \
rm -rf gpurun_out/prof_f && mkdir -p gpurun_out/prof_f && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f/trace_g -- python3 bench.py --workload global --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_f/tg.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_f/fetch_g -- python3 bench.py --workload global --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_f/fg.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_f/write_g -- python3 bench.py --workload global --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_f/wg.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_f/fetch_m -- python3 bench.py --workload mate --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_f/fm.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_f/write_m -- python3 bench.py --workload mate --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_f/wm.log 2>&1 && echo PROF_OK
for f in gpurun_out/bench_global.log gpurun_out/bench_mate.log; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['roofline']['launch_ms'], d['roofline']['frac'])"; done
