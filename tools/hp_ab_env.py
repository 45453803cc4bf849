"""Same-process A/B of a per-call environment switch of the host pipeline (GPU box): 1M-pair C2
bsw_get_scores calls alternating VAR unset / VAR=VALUE call by call (the library reads such
switches per call), after warm-up calls of both; prints median / q25 / min ms per setting.
usage: hp_ab_env.py VAR VALUE [calls per setting]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import hiprt  # noqa: E402,F401
import bsw  # noqa: E402

var, val = sys.argv[1], sys.argv[2]
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 20
pairs, ref, qer = bsw.synth_batch(1_000_000)
e = bsw.Engine()
want = pairs.copy()
e.get_scores(want, ref, qer, 100)
t = {"unset": [], val: []}
for k in range(2 * calls + 4):
    setting = "unset" if k % 2 == 0 else val
    if setting == "unset":
        os.environ.pop(var, None)
    else:
        os.environ[var] = val
    got = pairs.copy()
    t0 = time.perf_counter()
    e.get_scores(got, ref, qer, 100)
    ms = (time.perf_counter() - t0) * 1e3
    assert all(np.array_equal(got[f], want[f]) for f in bsw.OUT_FIELDS)
    if k >= 4:
        t[setting].append(ms)
for s, v in t.items():
    v = np.array(v)
    print(f"{var}={s}: median {np.median(v):.2f} q25 {np.percentile(v, 25):.2f} min {v.min():.2f} ms "
          f"({len(v)} calls) -> {1e3 / np.median(v):.1f} M pairs/s", flush=True)
