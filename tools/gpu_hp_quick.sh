#!/bin/bash
# host-buffer path: parity (chunked forms) + three ABI-inclusive measurements
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "host or chunk or guard or permuted" --timeout 250 --timeout-method thread > gpurun_out/hpq.log 2>&1; rc=$?
tail -2 gpurun_out/hpq.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_hpq.log 2>&1 && python -c "
import json; d=json.loads(open('gpurun_out/bench_hpq.log').read().strip().splitlines()[-1]); print(d['value'], d['abi_inclusive_value'], d['abi_inclusive']['ms_all_calls'], d['abi_inclusive']['last_call'])" || exit 1
done
