#!/bin/bash
# host-buffer pipeline: call time vs host worker count and max chunk
set -o pipefail
for t in 4 8 12 16; do
  echo "threads $t"; BSW_HOST_THREADS=$t timeout -k 10 120 python3 tools/host_path_once.py 262144 | tail -1
done
for c in 131072 524288; do
  echo "chunk $c"; timeout -k 10 120 python3 tools/host_path_once.py $c | tail -1
done
