#!/bin/bash
# rocprofv3 kernel trace + stats and the PMC passes (FETCH / WRITE / SQ / LDS) of the C2 bench on
# the final build (tools/profile.sh), for profiles/r03/final_prof.
set -o pipefail
OUT=gpurun_out/final_prof ARGS="--steps 20 --warmup 3 --no-cpu --no-host-path" bash tools/profile.sh > gpurun_out/final_prof.log 2>&1 || { tail -20 gpurun_out/final_prof.log; exit 1; }
tail -2 gpurun_out/final_prof.log
