#!/bin/bash
# 2-bit host staging check: host-path parity (chunked, packing forms), then two bench lines with
# the ABI-inclusive rate (2-bit) and the nibble staging beside it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "host or chunk or guard or permuted or packing" --timeout 250 --timeout-method thread > gpurun_out/hp2.log 2>&1; rc=$?
tail -2 gpurun_out/hp2.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_hp2.log 2>&1 && python -c "
import json; d=json.loads(open('gpurun_out/bench_hp2.log').read().strip().splitlines()[-1]); a=d['abi_inclusive']; print(d['value'], d['abi_inclusive_value'], a['ms_all_calls'], a['last_call'], a['nibble_staging'], json.dumps(a['per_call_curve']))" || exit 1
done
