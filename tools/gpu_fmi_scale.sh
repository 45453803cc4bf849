#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/fmi_scale
timeout -k 10 240 python -u -m pytest tests/test_fmi.py -m gpu -x -q -k "self_check or builder" --timeout 200 --timeout-method thread > gpurun_out/fmi_scale/tests.log 2>&1 || { tail -30 gpurun_out/fmi_scale/tests.log; exit 1; }
tail -2 gpurun_out/fmi_scale/tests.log
timeout -k 10 800 python -u tools/fmi_scale_check.py 200 1200 2200 3000 2>&1 | tee gpurun_out/fmi_scale/scale.log
