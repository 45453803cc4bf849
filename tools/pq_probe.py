"""Persistent host pipeline probe (GPU box): BSW_OPT_PERSIST 1 host-buffer calls on C2 pairs, each
call's stats (recovery step, launches, host / stage / kernel ms) and equality with the general
pipeline's outputs; BSW_DEBUG_HP=1 prints the eligibility and any failure of host_shard_pq."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import hiprt  # noqa: E402,F401
import bsw  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 4
only = os.environ.get("PQ_PROBE_ONCE")
pairs, ref, qer = bsw.synth_batch(1_000_000)
pairs = pairs[:n].copy()
base = bsw.Engine()
want = pairs.copy()
base.get_scores(want, ref, qer, 100)
for persist in ((1,) if only else (1, 0, 1)):
    e = bsw.Engine()
    e.set_option("persist", persist)
    for k in range(1 if only else calls):
        got = pairs.copy()
        t = time.perf_counter()
        e.get_scores(got, ref, qer, 100)
        ms = (time.perf_counter() - t) * 1e3
        st = e.last_stats()
        same = all(np.array_equal(got[f], want[f]) for f in bsw.OUT_FIELDS)
        print(f"persist {persist} call {k}: {ms:.2f} ms; host {st.host_ms:.2f} stage {st.stage_ms:.2f} "
              f"kernel {st.kernel_ms:.2f} launches {st.n_launches} recovery {st.recovery} same {same}", flush=True)
    e.close()
