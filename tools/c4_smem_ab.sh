set -o pipefail
O=gpurun_out/r6au; mkdir -p $O
for v in ${AB_VARIANTS:-base k3w6 k2w6 base k3w6 k2w6}; do
  if [ $v = base ]; then unset BSW_HIP_LIB; else export BSW_HIP_LIB=$PWD/bwa-mem2-arm_amd/lib/libbsw_hip_$v.so; fi
  timeout -k 10 300 python bench.py --workload c4mem --reads 10000000 --ref-mb 3000 --no-cpu --steps 6 --warmup 1 > $O/run.log 2>&1 || { echo "FAIL $v"; tail -5 $O/run.log; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('$O/run.log') if l.startswith('{')][-1]);print('$v', d['reads_per_s_M'], d['smem_kernel_ms'], d['stage_ms'])" | tee -a $O/c4ab.log
done
