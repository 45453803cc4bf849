#!/bin/bash
# Busy-routing parity under 8 callers; host pipeline chunk cap A/B (BSW_OPT_HOST_CHUNK 196608 /
# 262144 (default) / 524288), 10 calls per process, median of the last 7, x2.
set -o pipefail
O=gpurun_out/r3aa; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "busy_device or host_pipeline" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  line="rep $rep"
  for c in 196608 262144 524288; do
    timeout -k 10 200 python3 tools/host_path_once.py $c 10 > $O/hp_${c}_$rep.log 2>&1 || { tail $O/hp_${c}_$rep.log; exit 1; }
    med=$(grep '^call' $O/hp_${c}_$rep.log | tail -7 | awk '{print $2}' | sort -n | sed -n 4p)
    line="$line | chunk $c median $med ms"
  done
  echo "$line"
done
