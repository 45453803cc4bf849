#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_batch_file.py tests/test_ext_pipeline.py tests/test_dist_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_d.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python tools/host_chunk_sweep.py > gpurun_out/chunk_sweep.log 2>&1 && echo SWEEP_OK && cat gpurun_out/chunk_sweep.log && \
rm -rf gpurun_out/hptrace && \
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hptrace -- python3 tools/host_path_once.py 262144 > gpurun_out/hptrace.log 2>&1 && echo TRACE_OK && grep call gpurun_out/hptrace.log
