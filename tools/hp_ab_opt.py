"""Same-process A/B of an engine option on the host pipeline (GPU box): two engines, one at the
default and one with OPTION=VALUE, alternating 1M-pair C2 bsw_get_scores calls after warm-up calls
of both; prints median / q25 / min ms per engine.  usage: hp_ab_opt.py OPTION VALUE [calls]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import hiprt  # noqa: E402,F401
import bsw  # noqa: E402

opt, val = sys.argv[1], int(sys.argv[2])
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 20
pairs, ref, qer = bsw.synth_batch(1_000_000)
a, b = bsw.Engine(), bsw.Engine()
b.set_option(opt, val)
want = pairs.copy()
a.get_scores(want, ref, qer, 100)
t = {"default": [], f"{opt}={val}": []}
for k in range(2 * calls + 4):
    e, tag = (a, "default") if k % 2 == 0 else (b, f"{opt}={val}")
    got = pairs.copy()
    t0 = time.perf_counter()
    e.get_scores(got, ref, qer, 100)
    ms = (time.perf_counter() - t0) * 1e3
    assert all(np.array_equal(got[f], want[f]) for f in bsw.OUT_FIELDS)
    if k >= 4:
        t[tag].append(ms)
for s, v in t.items():
    v = np.array(v)
    print(f"{s}: median {np.median(v):.2f} q25 {np.percentile(v, 25):.2f} min {v.min():.2f} ms ({len(v)} calls) "
          f"-> {1e3 / np.median(v):.1f} M pairs/s", flush=True)
