"""A/B timing of library variants (timing only, interleaved rounds in ONE process per variant set)."""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'bwa-mem2-arm_amd', 'py'))
import hiprt, bsw
libs = sys.argv[1:]
pairs, ref, qer = bsw.synth_batch(1_000_000)
dp = hiprt.DeviceBuffer.from_array(pairs); dr = hiprt.DeviceBuffer.from_array(ref); dq = hiprt.DeviceBuffer.from_array(qer)
engines = []
for path in libs:
    L = ctypes.CDLL(os.path.abspath(path))
    P = ctypes.c_void_p
    L.bsw_create.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(P)]
    L.bsw_get_scores_device.argtypes = [P, P, P, P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int, P]
    L.bsw_last_stats.argtypes = [P, P]
    ctx = P(); prm = bsw.default_params()
    assert L.bsw_create(ctypes.byref(prm), 0, 1, ctypes.byref(ctx)) == 0
    engines.append((path, L, ctx))
res = {p: [] for p, _, _ in engines}
for rnd in range(6):
    for path, L, ctx in engines:
        rc = L.bsw_get_scores_device(ctx, P(dp.ptr), P(dr.ptr), P(dq.ptr), len(pairs), 100, 16, None)
        st = bsw.Stats(); L.bsw_last_stats(ctx, ctypes.byref(st))
        if rnd: res[path].append(st.kernel_ms)
for p, v in res.items():
    print(f"{os.path.basename(p):28s} kernel ms median {np.median(v):8.3f} min {min(v):8.3f}")
