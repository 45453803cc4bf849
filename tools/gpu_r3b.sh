#!/bin/bash
# Round 3: the seeding -> chaining -> extension front end on the GPU (tests/test_memchain.py).
set -o pipefail
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest tests/test_memchain.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3b/memchain.log 2>&1 || { tail -40 gpurun_out/r3b/memchain.log; exit 1; }
tail -8 gpurun_out/r3b/memchain.log
