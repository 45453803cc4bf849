"""Cross-call coalescing probe: 8 concurrent callers of m-pair host-buffer calls (C2 shape);
per call the batch it ran in (pairs), its host / staging / DP-kernel ms; the aggregate rate.
Run under rocprofv3 --kernel-trace to see the GPU timeline."""
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import hiprt  # noqa: E402,F401
import bsw  # noqa: E402

pairs, ref, qer = bsw.synth_batch(400_000)
for co, lead in ((32768, 2), (32768, 3), (32768, 4), (32768, 6), (0, 1)):
    e = bsw.Engine(coalesce=co, coalesce_leaders=lead)
    for m in (1000, 10000):
        per = 40 if m == 1000 else 12
        recs = []
        lock = threading.Lock()
        go = threading.Barrier(9)

        def worker(k):
            e.get_scores(pairs[:m].copy(), ref, qer, 100)
            go.wait()
            go.wait()
            for c in range(per):
                a = ((k * per + c) * m) % (len(pairs) - m)
                v = pairs[a:a + m].copy()
                t = time.perf_counter()
                e.get_scores(v, ref, qer, 100)
                dt = time.perf_counter() - t
                st = e.last_stats()
                with lock:
                    recs.append((dt * 1e3, st.n_i16 + st.n_u8 + st.n_wide, st.host_ms, st.stage_ms, st.kernel_ms))
        th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
        for x in th:
            x.start()
        go.wait()
        t = time.perf_counter()
        go.wait()
        for x in th:
            x.join()
        dt = time.perf_counter() - t
        med = lambda i: statistics.median(r[i] for r in recs)  # noqa: E731
        print(f"coalesce {co:6d} leaders {lead} m {m:6d}: {8 * per * m / dt / 1e6:7.2f} M/s; per call median: wall {med(0):.3f} ms, "
              f"batch {med(1):.0f} pairs, host {med(2):.3f} ms, stage {med(3):.3f} ms, dp kernel {med(4):.3f} ms",
              flush=True)
    e.close()
