set -e
for k in 1 2; do
for v in 2 4; do BSW_SORTKEY=$v timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/ab_$v.log 2>&1; echo "KEY=$v $(python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['launch_ms'])")"; done
done
