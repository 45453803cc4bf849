#!/bin/bash
# Round-3 closing lines of the secondary BASELINE configs on the final build: C1 (the reference's
# own 10K reads vs 1 Mb), C4 front end at 1M / 64 Mb and at BASELINE scale (10M PE vs 3 Gb).
set -o pipefail
O=gpurun_out/final3c; mkdir -p $O
timeout -k 10 300 python -u bench.py --workload c1 --steps 10 --warmup 2 > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
tail -1 $O/c1.log | cut -c1-300
timeout -k 10 400 python -u bench.py --workload c4mem --reads 1000000 --ref-mb 64 --steps 5 --warmup 1 > $O/c4_64.log 2>&1 || { tail -20 $O/c4_64.log; exit 1; }
tail -1 $O/c4_64.log | cut -c1-300
timeout -k 10 900 python -u bench.py --workload c4mem --reads 10000000 --ref-mb 3000 --steps 3 --warmup 1 > $O/c4_3gb.log 2>&1 || { tail -20 $O/c4_3gb.log; exit 1; }
tail -1 $O/c4_3gb.log | cut -c1-300
