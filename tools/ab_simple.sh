set -e
for k in 1 2 3; do timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/ab.log 2>&1; python3 -c "import json;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['launch_ms'])"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1
