#!/bin/bash
# Round-2 refresh: full GPU suite, default bench line, rocprofv3 passes (summarised on the box),
# secondary bench lines.  Everything lands in gpurun_out/r02/.
set -o pipefail
mkdir -p gpurun_out/r02
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r02/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r02/bench.log 2>&1 || exit 1
OUT=gpurun_out/prof bash tools/profile.sh || exit 1
python tools/pmc_summary.py gpurun_out/prof gpurun_out/r02/sum > gpurun_out/r02/pmc.txt 2>&1
cp profiles/pmc_latest.json gpurun_out/r02/sum/pmc_latest.json
find gpurun_out/prof -type f -size +2M -delete
for w in mate global; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 > gpurun_out/r02/bench_$w.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --cell-bits 8 --h0-hi 130 --no-cpu --no-host-path > gpurun_out/r02/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c4seed --steps 3 --warmup 1 > gpurun_out/r02/bench_c4seed.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c1 --steps 5 --warmup 1 > gpurun_out/r02/bench_c1.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload smem --steps 3 --warmup 1 > gpurun_out/r02/bench_smem.log 2>&1 || exit 1
for f in gpurun_out/r02/bench*.log; do echo "$f $(tail -1 $f | cut -c1-150)"; done
echo refresh-done
