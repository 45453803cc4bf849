"""Host-path fast-path timeline (experiment; GPU box): BSW_DEBUG_HP=1 per-chunk host timings of a
few 1M-pair C2 bsw_get_scores calls, plus each call's last_stats (host / stage / kernel ms)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import hiprt  # noqa: E402,F401
import bsw  # noqa: E402

pairs, ref, qer = bsw.synth_batch(1_000_000)
e = bsw.Engine()
buf = pairs.copy()
for k in range(4):
    t = time.perf_counter()
    e.get_scores(buf, ref, qer, 100)
    st = e.last_stats()
    print(f"call {k}: {(time.perf_counter() - t) * 1e3:.2f} ms; host {st.host_ms:.2f} stage {st.stage_ms:.2f} "
          f"kernels {st.kernel_ms:.2f} launches {st.n_launches}", file=sys.stderr, flush=True)
