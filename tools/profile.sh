#!/bin/bash
# rocprofv3 passes over a short bench run (run ON the GPU box, from the repo root).
#   1. kernel trace + stats        -> gpurun_out/prof/trace
#   2. PMC FETCH_SIZE              -> gpurun_out/prof/pmc_fetch
#   3. PMC WRITE_SIZE              -> gpurun_out/prof/pmc_write
#   4. PMC SQ occupancy/VALU       -> gpurun_out/prof/pmc_sq
#   5. PMC LDS bank conflicts + L2 hit/miss -> gpurun_out/prof/pmc_lds
# Counters are collected in their own passes with --kernel-trace only (never with
# sys/runtime traces).  Every pass runs under its own timeout; any failure stops the script.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=${OUT:-gpurun_out/prof}
ARGS=${ARGS:---steps 5 --warmup 1 --no-cpu --no-host-path}
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -- python3 bench.py $ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -- python3 bench.py $ARGS > "$OUT/pmc_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --output-format csv -d "$OUT/pmc_sq" -- python3 bench.py $ARGS > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_lds" -- python3 bench.py $ARGS > "$OUT/pmc_lds.log" 2>&1
echo profile-done
