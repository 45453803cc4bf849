#!/bin/bash
# Chain / extension tests after the scratch cache + retry-readback fold, the C1 line, then the
# host-buffer A/B (in-tree library vs lib/libbsw_hip_base.so).
set -o pipefail
mkdir -p gpurun_out/r3i
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_chain.py tests/test_memchain.py tests/test_ext_pipeline.py tests/test_fmi.py > gpurun_out/r3i/tests.log 2>&1 || { tail -30 gpurun_out/r3i/tests.log; exit 1; }
tail -1 gpurun_out/r3i/tests.log
timeout -k 10 200 python bench.py --workload c1 --steps 10 --warmup 2 > gpurun_out/r3i/c1.log 2>&1 || { tail -5 gpurun_out/r3i/c1.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r3i/c1.log').read().strip().splitlines()[-1]);print('c1', d['value'], d['ms_per_step'], d['stage_ms'])"
bash tools/gpu_ab_host.sh
