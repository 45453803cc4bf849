#!/bin/bash
# SMEM kernel: bench line + kernel trace + FETCH/WRITE passes (one launch per call)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P=gpurun_out/prof_s
rm -rf $P; mkdir -p $P gpurun_out/r02s
A="--workload smem --steps 2 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -- python3 bench.py $A > $P/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -- python3 bench.py $A > $P/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -- python3 bench.py $A > $P/write.log 2>&1 || exit 1
python tools/pmc_summary.py $P gpurun_out/r02s/sum > gpurun_out/r02s/pmc.txt 2>&1
find $P -type f -size +2M -delete
timeout -k 10 400 python bench.py --workload smem --steps 3 --warmup 1 > gpurun_out/r02s/bench_smem.log 2>&1 || exit 1
tail -1 gpurun_out/r02s/bench_smem.log | cut -c1-200
