#!/bin/bash
# timeline of the host-buffer pipeline: kernel + memory-copy trace of 3 host-buffer calls (1M C2 pairs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf gpurun_out/hp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hp -- python3 tools/host_path_once.py > gpurun_out/hp_trace.log 2>&1
rc=$?
tail -5 gpurun_out/hp_trace.log
find gpurun_out/hp -name '*.csv' | head
exit $rc
