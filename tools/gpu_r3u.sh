#!/bin/bash
# NOTE: the BSW_HP_NO_EARLY / BSW_HP_NO_MERGE switches were removed with the variants after this A/B.
# Host-buffer pipeline A/B (1M C2 pairs, pageable buffers): early start (first chunk's prepass only,
# the rest after chunk 0 is enqueued) and the remainder chunk merged, against each switched off
# (BSW_HP_NO_EARLY / BSW_HP_NO_MERGE, experiment switches); interleaved x3, 3 calls each (the
# first is warm-up), per-chunk timeline kept.
set -o pipefail
O=gpurun_out/r3u; mkdir -p $O
for rep in 1 2 3; do
  line="rep $rep"
  for v in new noearly nomerge old; do
    case $v in new) E="";; noearly) E="BSW_HP_NO_EARLY=1";; nomerge) E="BSW_HP_NO_MERGE=1";; old) E="BSW_HP_NO_EARLY=1 BSW_HP_NO_MERGE=1";; esac
    timeout -k 10 200 env BSW_DEBUG_HP=1 $E python3 tools/host_path_once.py > $O/${v}_$rep.log 2>&1 || { tail $O/${v}_$rep.log; exit 1; }
    line="$line | $v: $(grep '^call' $O/${v}_$rep.log | tail -2 | cut -c6-14 | tr '\n' ' ')"
  done
  echo "$line"
done
tail -9 $O/new_3.log
