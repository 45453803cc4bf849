#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3j
timeout -k 10 400 python bench.py > gpurun_out/r3j/bench.log 2> gpurun_out/r3j/bench.err || { tail -20 gpurun_out/r3j/bench.err; exit 1; }
tail -1 gpurun_out/r3j/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); a=d.get('abi_inclusive',{})
print('value',d['value'],'abi',d.get('abi_inclusive_value'),'frac',d['roofline']['frac'],'ms',d['ms_per_step'])
for k in ('per_call_curve','per_call_curve_without_coalescing','per_call_curve_cpp_callers'):
    print(k, json.dumps(a.get(k))[:1500])
print('cpu', json.dumps(d['cpu_baseline'])[:800])"
