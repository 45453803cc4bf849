#!/bin/bash
# Round-3 PMC passes on the secondary kernels: the wave kernel (250-bp reads), the row-group
# small-batch kernel (16K C2 pairs per device call) and the SMEM kernel (16 Mb index).
# Each workload: kernel trace + FETCH_SIZE + WRITE_SIZE + SQ passes, each under its own timeout.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() {
  local tag=$1; shift
  OUT=gpurun_out/pmc3/$tag ARGS="$*" bash tools/profile.sh > gpurun_out/pmc3/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/pmc3/$tag.log; exit 1; }
  echo "done $tag"
}
mkdir -p gpurun_out/pmc3
run wv --qlen 250 --tlen 350 --pairs 500000 --steps 3 --warmup 1 --no-cpu --no-host-path
run gq --pairs 16000 --steps 20 --warmup 2 --no-cpu --no-host-path
run smem --workload smem --reads 1000000 --steps 3 --warmup 1 --no-cpu
