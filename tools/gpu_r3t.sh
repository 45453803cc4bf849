#!/bin/bash
# Host-buffer pipeline: per-chunk host timeline (BSW_DEBUG_HP) of 1M-pair calls, untraced.
set -o pipefail
mkdir -p gpurun_out/r3t
timeout -k 10 200 env BSW_DEBUG_HP=1 python3 tools/host_path_once.py > gpurun_out/r3t/hp.log 2>&1 || { tail gpurun_out/r3t/hp.log; exit 1; }
tail -30 gpurun_out/r3t/hp.log
