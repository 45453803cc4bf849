#!/bin/bash
# Text-mode SMEM walk: parity (FM-index, chaining, front end), then same-box A/B at 16 Mb (smem)
# and 64 Mb (C4 front end) with and without the text-mode data.
set -o pipefail
mkdir -p gpurun_out/r3l
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_fmi.py tests/test_memchain.py tests/test_chain.py > gpurun_out/r3l/tests.log 2>&1 || { tail -40 gpurun_out/r3l/tests.log; exit 1; }
tail -1 gpurun_out/r3l/tests.log
for k in 1 2; do for v in text blocks; do
  F=""; [ $v = blocks ] && F="--fmi-blocks-only"
  timeout -k 10 200 python bench.py --workload smem --steps 5 --warmup 1 --no-cpu $F > gpurun_out/r3l/smem_$v.log 2>&1 || { tail -5 gpurun_out/r3l/smem_$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r3l/smem_$v.log').read().strip().splitlines()[-1]);print('smem $v', d['value'], d['ms_per_step'])"
done; done
for v in text blocks; do
  F=""; [ $v = blocks ] && F="--fmi-blocks-only"
  timeout -k 10 300 python bench.py --workload c4mem --steps 5 --warmup 1 --no-cpu $F > gpurun_out/r3l/c4mem_$v.log 2> gpurun_out/r3l/c4mem_$v.err || { tail -5 gpurun_out/r3l/c4mem_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r3l/c4mem_$v.log').read().strip().splitlines()[-1]);print('c4mem $v', d['value'], d['reads_per_s_M'], d['stage_ms'])"
done
