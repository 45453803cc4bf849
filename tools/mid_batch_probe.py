"""Device-call time of C2 batches of 4K..128K pairs on the row-group kernel (16 lanes / quads)
vs the planned lane-kernel path (BSW_OPT_GROUP_KERNEL 0): median of 9 calls, event-timed DP."""
import os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import numpy as np
import bsw, hiprt

pairs, ref, qer = bsw.synth_batch(131072)
dr, dq = hiprt.DeviceBuffer.from_array(ref), hiprt.DeviceBuffer.from_array(qer)
engines = {"rowgroup": bsw.Engine(), "rowgroup16 only": bsw.Engine(mid_batch=0), "planned": bsw.Engine(group_kernel=0),
           "quads only": bsw.Engine(small_batch=0, mid_batch=131072)}
for n in (4096, 16384, 24576, 32768, 49152, 65536, 131072):
    dp = hiprt.DeviceBuffer.from_array(pairs[:n].copy())
    row = []
    for name, e in engines.items():
        ts, ks = [], []
        for _ in range(10):
            t = time.perf_counter()
            e.get_scores_device(dp.ptr, dr.ptr, dq.ptr, n, 100, 16)
            ts.append(time.perf_counter() - t)
            ks.append(e.last_stats().kernel_ms)
        st = e.last_stats()
        row.append(f"{name}: {statistics.median(ts[1:])*1e3:.3f} ms (kernel {statistics.median(ks[1:]):.3f}, grp {st.n_group})")
    print(f"n={n:6d}  " + " | ".join(row), flush=True)
