#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/list_avail.log 2>&1; echo LIST_RC=$?
OUT=gpurun_out/prof bash tools/profile.sh && echo PROF_OK
