"""Per-call latency of small host-buffer batches (C2 shape) under the default routing
(lane / packed-column kernels) and with every pair on the wave-per-alignment kernel
(BSW_OPT_LONG = 2): median of 20 calls after warm-up, from one caller."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import hiprt  # noqa: E402,F401
import bsw  # noqa: E402

pairs, ref, qer = bsw.synth_batch(200_000)
for route in (1, 2):
    e = bsw.Engine(long=route)
    for m in (256, 1000, 4000, 10000, 30000, 100000):
        buf = pairs[:m].copy()
        for _ in range(3):
            e.get_scores(buf, ref, qer, 100)
        ts = []
        for k in range(20):
            v = pairs[(k * m) % (len(pairs) - m):][:m].copy()
            t = time.perf_counter()
            e.get_scores(v, ref, qer, 100)
            ts.append(time.perf_counter() - t)
        st = e.last_stats()
        print(f"route {route} pairs {m:6d} call_ms {statistics.median(ts) * 1e3:7.3f} kernel_ms {st.kernel_ms:7.3f} "
              f"n_wave {st.n_wave} n_packed {st.n_packed}", flush=True)
    e.close()
