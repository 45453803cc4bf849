#!/bin/bash
# SMEM kernel lane utilisation (divergence): thread-cycles vs instruction-cycles of VALU.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/pmcdiv
timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcdiv/p1 -- python3 bench.py --workload smem --steps 2 --warmup 1 --no-cpu > gpurun_out/pmcdiv/p1.log 2>&1 || { tail -5 gpurun_out/pmcdiv/p1.log; exit 1; }
python3 - <<'PY'
import csv,glob,collections
acc=collections.defaultdict(list)
for f in glob.glob('gpurun_out/pmcdiv/p1/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'smem_kernel' in r['Kernel_Name']:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
for k,v in acc.items(): print(k, sum(v)/len(v))
t=acc.get('SQ_THREAD_CYCLES_VALU'); a=acc.get('SQ_ACTIVE_INST_VALU')
if t and a: print('lane utilisation ~', (sum(t)/len(t))/(64*sum(a)/len(a)))
PY
