"""C3 study (BASELINE configs[2]): the 8-bit-regime kernel + int16 overflow fallback on gfx950.

Runs on the GPU box.  For the C2 batch shape with h0 ~ U[19, H0HI] (H0HI = 105: every pair in
the 8-bit regime; 130 / 160: a measurable int16 fallback fraction) and both entry points
(cell_bits 8 = getScores8, 16 = getScores16) it records the routing (n_u8 / n_i16 / n_packed),
the DP kernel time and the step time; with BSW_OPT_KERNEL8 = 0 the same batch on the int16 lane
kernel only.  Writes one JSON document to stdout (profiles/r02/c3_study.json)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import numpy as np  # noqa: E402
import hiprt  # noqa: E402
import bsw  # noqa: E402

N = 1_000_000
out = {"pairs": N, "shape": "150 bp query / 300 bp ref, w=100, bwa defaults", "runs": []}
for h0hi in (105, 130, 160):
    cfg = bsw.synth_cfg(h0_hi=h0hi)
    pairs, ref, qer = bsw.synth_batch(N, cfg=cfg)
    dp, dr, dq = (hiprt.DeviceBuffer.from_array(a) for a in (pairs, ref, qer))
    for kernel8 in (1, 0):
        eng = bsw.Engine(kernel8=kernel8)
        for cb in ((8, 16) if kernel8 else (16,)):
            for _ in range(2):
                eng.get_scores_device(dp.ptr, dr.ptr, dq.ptr, N, 100, cb)
            ts, ks = [], []
            for _ in range(5):
                hiprt.synchronize()
                t = time.perf_counter()
                eng.get_scores_device(dp.ptr, dr.ptr, dq.ptr, N, 100, cb)
                ts.append(time.perf_counter() - t)
                ks.append(eng.last_stats().kernel_ms)
            st = eng.last_stats()
            step = float(np.median(ts))
            out["runs"].append({
                "h0": [19, h0hi], "cell_bits": cb, "kernel8": kernel8,
                "routing": {"n_packed": st.n_packed, "n_u8": st.n_u8, "n_i16": st.n_i16, "n_wide": st.n_wide,
                            "launches": st.n_launches},
                "int16_fallback_fraction": round(st.n_i16 / N, 4) if cb == 8 else None,
                "dp_kernel_ms": round(float(np.median(ks)), 3), "step_ms": round(step * 1e3, 3),
                "M_pairs_per_s": round(N / step / 1e6, 2)})
            print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
        eng.close()
print(json.dumps(out, indent=1))
