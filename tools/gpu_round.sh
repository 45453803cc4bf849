set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench.log && \
OUT=gpurun_out/prof bash tools/profile.sh
