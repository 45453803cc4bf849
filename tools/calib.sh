#!/bin/bash
# FETCH_SIZE calibration pass (GPU box, repo root): known-byte kernels under rocprofv3.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=${OUT:-gpurun_out/calib}
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -- ./tools/fetch_calib > "$OUT/fetch.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -- ./tools/fetch_calib > "$OUT/write.log" 2>&1
echo calib-done
