# class-launch fork check: GPU tests, then C1 / C4 / C2 with and without the fork
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -1 gpurun_out/gpu_tests.log
for v in fork nofork; do
  if [ $v = nofork ]; then export BSW_NO_FORK=1; fi
  for wl in c1 c4 c2; do
    timeout -k 10 300 python bench.py --workload $wl --no-cpu --steps 5 --warmup 1 > gpurun_out/fork_${v}_$wl.log 2>&1
    echo "$v $wl $(python3 -c "import json;d=json.loads(open('gpurun_out/fork_${v}_$wl.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
