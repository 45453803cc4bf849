"""Host-buffer bsw_get_scores calls over the 1M C2 batch, one line per call (first-call cost and
timeline traces).  argv: chunk pairs (262144), calls (3), 1 = a resident device call first (as
bench.py runs before its host-path leg)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import hiprt  # noqa: E402,F401
import bsw  # noqa: E402

chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
pairs, ref, qer = bsw.synth_batch(1_000_000)
e = bsw.Engine(host_chunk=chunk)
if len(sys.argv) > 3 and sys.argv[3] == "1":
    d = [hiprt.DeviceBuffer.from_array(a) for a in (pairs, ref, qer)]
    for _ in range(3):
        e.get_scores_device(d[0].ptr, d[1].ptr, d[2].ptr, len(pairs), 100, 16)
buf = pairs.copy()
for _ in range(calls):
    t = time.perf_counter()
    e.get_scores(buf, ref, qer, 100)
    st = e.last_stats()
    print(f"call {(time.perf_counter() - t) * 1e3:.2f} ms host {st.host_ms:.2f} stage {st.stage_ms:.2f} "
          f"kernels {st.kernel_ms:.2f} launches {st.n_launches}", flush=True)
