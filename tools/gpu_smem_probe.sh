#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 500 python -u tools/smem_phase_probe.py 1000 2000000 2>&1 | tee gpurun_out/probe/smem_phases.txt
