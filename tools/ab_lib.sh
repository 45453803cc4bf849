# A/B of two product builds on one box: the in-tree library vs lib/libbsw_hip_base.so
set -e
for k in 1 2; do
for v in base new; do
  if [ $v = base ]; then export BSW_HIP_LIB=$PWD/bwa-mem2-arm_amd/lib/libbsw_hip_base.so; else unset BSW_HIP_LIB; fi
  timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/ab_$v.log 2>&1
  echo "$v $(python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['launch_ms'])")"
done
done
unset BSW_HIP_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2
