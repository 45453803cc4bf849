#!/bin/bash
# C2 bench line + rocprofv3 passes, summarised ON the box (raw traces are too large to merge back).
#   gpurun_out/r02/bench.log        the default bench line
#   gpurun_out/r02/sum/             kernel_stats.csv + pmc_summary.json (tools/pmc_summary.py)
set -euo pipefail
mkdir -p gpurun_out/r02
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python bench.py > gpurun_out/r02/bench.log 2>&1
tail -1 gpurun_out/r02/bench.log | cut -c1-300
OUT=gpurun_out/prof bash tools/profile.sh
python tools/pmc_summary.py gpurun_out/prof gpurun_out/r02/sum > gpurun_out/r02/pmc.txt 2>&1
cp profiles/pmc_latest.json gpurun_out/r02/sum/pmc_latest.json
find gpurun_out/prof -type f -size +2M -delete
echo prof-done
