"""Host-buffer pipeline chunk-size sweep (BSW_OPT_HOST_CHUNK) on the 1M C2 batch."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import hiprt  # noqa: E402,F401
import bsw  # noqa: E402

pairs, ref, qer = bsw.synth_batch(1_000_000)
for chunk in [int(x) for x in sys.argv[1:]] or (65536, 131072, 262144, 524288, 1_000_000):
    e = bsw.Engine(host_chunk=chunk)
    buf = pairs.copy()
    e.get_scores(buf, ref, qer, 100)
    ts = []
    for _ in range(6):
        t = time.perf_counter()
        e.get_scores(buf, ref, qer, 100)
        ts.append(time.perf_counter() - t)
    st = e.last_stats()
    print(json.dumps({"chunk": chunk, "ms": round(min(ts) * 1e3, 2), "ms_median": round(sorted(ts)[len(ts) // 2] * 1e3, 2), "M_pairs_s": round(1e6 / min(ts) / 1e6 * 1e0, 2),
                      "stage_ms": round(st.stage_ms, 2), "host_ms": round(st.host_ms, 2),
                      "kernel_ms": round(st.kernel_ms, 2)}), flush=True)
    e.close()
