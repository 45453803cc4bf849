"""Host-buffer path probe (experiment; GPU box): C2 1M-pair bsw_get_scores calls after a warm-up,
median / min wall ms and M pairs/s, outputs checked against the resident call; plus the resident
call's DP kernel ms (the LDS-padding experiments: BSW_HP_LDS_PAD / BSW_PC_LDS_PAD in the env).
  python tools/hp_probe.py [calls]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import numpy as np  # noqa: E402
import hiprt  # noqa: E402
import bsw  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 10
pairs, ref, qer = bsw.synth_batch(1_000_000)
e = bsw.Engine()
d = [hiprt.DeviceBuffer.from_array(a) for a in (pairs, ref, qer)]
km = []
for k in range(6):
    e.get_scores_device(d[0].ptr, d[1].ptr, d[2].ptr, len(pairs), 100)
    km.append(e.last_stats().kernel_ms)
want = d[0].download(np.empty_like(pairs))
buf = pairs.copy()
ms = []
for k in range(calls + 2):
    t = time.perf_counter()
    e.get_scores(buf, ref, qer, 100)
    if k >= 2:
        ms.append((time.perf_counter() - t) * 1e3)
same = all(np.array_equal(buf[f], want[f]) for f in bsw.OUT_FIELDS)
med = statistics.median(ms)
print(f"fast={os.environ.get('BSW_HP_FAST', '-')} pads hp={os.environ.get('BSW_HP_LDS_PAD', '-')} pc={os.environ.get('BSW_PC_LDS_PAD', '-')}: host call median "
      f"{med:.2f} ms (min {min(ms):.2f}) = {1e3 / med:.1f} M/s; resident DP kernel {statistics.median(km[2:]):.3f} ms; "
      f"outputs identical {same}; calls {[round(x, 2) for x in ms]}", flush=True)
