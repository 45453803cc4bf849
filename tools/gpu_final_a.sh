#!/bin/bash
# Round-2 final refresh, part A: full GPU suite, default C2 bench line (CPU baseline + host path),
# rocprofv3 passes summarised on the box.  Output: gpurun_out/r02/
set -o pipefail
mkdir -p gpurun_out/r02
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r02/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r02/bench.log 2>&1 || exit 1
tail -c 600 gpurun_out/r02/bench.log; echo
OUT=gpurun_out/prof bash tools/profile.sh || exit 1
python tools/pmc_summary.py gpurun_out/prof gpurun_out/r02/sum > gpurun_out/r02/pmc.txt 2>&1
cp profiles/pmc_latest.json gpurun_out/r02/sum/pmc_latest.json
find gpurun_out/prof -type f -size +2M -delete
echo final-a-done
