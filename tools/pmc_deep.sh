#!/bin/bash
# Deeper SQ/SQC counter passes on a short bench run (GPU box, repo root).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=${OUT:-gpurun_out/deep}
ARGS=${ARGS:---steps 2 --warmup 1 --no-cpu --no-host-path}
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU --output-format csv -d "$OUT/a" -- python3 bench.py $ARGS > "$OUT/a.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VSKIPPED --output-format csv -d "$OUT/b" -- python3 bench.py $ARGS > "$OUT/b.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ GRBM_GUI_ACTIVE --output-format csv -d "$OUT/c" -- python3 bench.py $ARGS > "$OUT/c.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VALU2 SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM --output-format csv -d "$OUT/d" -- python3 bench.py $ARGS > "$OUT/d.log" 2>&1
echo deep-done
