#!/bin/bash
# Round-3 closing check of the committed tree: whole GPU suite, smoke(), default bench line.
set -o pipefail
O=gpurun_out/final3b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['launch_ms'], d['roofline']['frac'], d['abi_inclusive_value'], d['cpu_baseline']['value'], [(c['pairs_per_call'], c['coalescing'], c['M_pairs_per_s_8_callers']) for c in d['abi_inclusive']['per_call_curve_cpp_callers']['curve']])"
