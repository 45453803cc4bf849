#!/bin/bash
# PMC HBM-traffic passes for the (f)-row kernels: global (+CIGAR), mate rescue, SMEM seeding.
# Separate --pmc runs (kernel trace + stats in their own run); summary on the box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P=gpurun_out/prof_f
rm -rf $P; mkdir -p $P
for w in global mate smem; do
  A="--workload $w --steps 2 --warmup 1 --no-cpu"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/$w/trace -- python3 bench.py $A > $P/$w.trace.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/$w/fetch -- python3 bench.py $A > $P/$w.fetch.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/$w/write -- python3 bench.py $A > $P/$w.write.log 2>&1 || exit 1
  echo "$w done"
done
mkdir -p gpurun_out/r02f
python tools/pmc_summary.py $P gpurun_out/r02f/sum > gpurun_out/r02f/pmc.txt 2>&1
find $P -type f -size +2M -delete
echo pmc-frows-done
