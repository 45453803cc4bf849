#!/bin/bash
# Text-mode SMEM walk at BASELINE scale: C4 front end, 10M PE reads vs 3 Gb, with and without.
set -o pipefail
mkdir -p gpurun_out/r3m
for v in text blocks; do
  F=""; [ $v = blocks ] && F="--fmi-blocks-only"
  timeout -k 10 500 python bench.py --workload c4mem --reads 10000000 --ref-mb 3000 --steps 3 --warmup 1 --no-cpu $F > gpurun_out/r3m/c4mem3g_$v.log 2> gpurun_out/r3m/c4mem3g_$v.err || { tail -5 gpurun_out/r3m/c4mem3g_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r3m/c4mem3g_$v.log').read().strip().splitlines()[-1]);print('c4mem3g $v', d['value'], d['reads_per_s_M'], d['stage_ms'], d['index'])"
done
