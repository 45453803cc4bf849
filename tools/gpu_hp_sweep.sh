#!/bin/bash
# host-buffer call time vs the pipeline's largest chunk (3 calls each, after one warm call)
set -o pipefail
for c in 196608 262144 393216 524288; do
  echo "chunk $c"; timeout -k 10 120 python3 tools/host_path_once.py $c | tail -2 || exit 1
done
