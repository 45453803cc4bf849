"""One host-buffer bsw_get_scores over the 1M C2 batch (after a warm-up) for timeline traces."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import hiprt  # noqa: E402,F401
import bsw  # noqa: E402

chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
pairs, ref, qer = bsw.synth_batch(1_000_000)
e = bsw.Engine(host_chunk=chunk)
buf = pairs.copy()
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    t = time.perf_counter()
    e.get_scores(buf, ref, qer, 100)
    st = e.last_stats()
    print(f"call {(time.perf_counter() - t) * 1e3:.2f} ms host {st.host_ms:.2f} stage {st.stage_ms:.2f} "
          f"kernels {st.kernel_ms:.2f}", flush=True)
