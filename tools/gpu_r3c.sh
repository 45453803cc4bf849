#!/bin/bash
# Round 3: cross-call coalescing -- its parity test, the small-call tests, then the C2 bench
# line (per-call curve with and without coalescing, same box).
set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "coalesced or small_batch or concurrent or multi_device or host_pipeline" --timeout 300 --timeout-method thread > gpurun_out/r3c/tests.log 2>&1 || { tail -40 gpurun_out/r3c/tests.log; exit 1; }
tail -4 gpurun_out/r3c/tests.log
timeout -k 10 400 python bench.py > gpurun_out/r3c/bench.log 2>&1 || { tail -30 gpurun_out/r3c/bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r3c/bench.log") if l.startswith("{")][-1])
a = d["abi_inclusive"]
print("value", d["value"], "abi", d["abi_inclusive_value"])
print("curve", a["per_call_curve"])
print("no-coalesce", a["per_call_curve_without_coalescing"])
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"].get("node_extrapolated"))
PY
