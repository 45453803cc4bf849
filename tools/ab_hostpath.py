"""Interleaved same-process A/B of the host-buffer (drop-in) path between two builds of the
product library: calls alternate A, B, A, B ... on the same 1M C2 pairs, so the box's varying
host-memory bandwidth hits both alike.  usage: python tools/ab_hostpath.py LIB_A LIB_B [reps]"""
import ctypes, os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import numpy as np
import bsw

reps = int(sys.argv[3]) if len(sys.argv) > 3 else 15
# optional per-library host pool sizes (BSW_HOST_THREADS, read when a library's pool starts)
threads = sys.argv[4:6] if len(sys.argv) > 5 else None
libs = [ctypes.CDLL(p) for p in sys.argv[1:3]]
pairs, ref, qer = bsw.synth_batch(1_000_000)
params = bsw.default_params()
ctxs = []
for L in libs:
    c = ctypes.c_void_p()
    assert L.bsw_create(ctypes.byref(params), 0, 1, ctypes.byref(c)) == 0
    ctxs.append(c)
P = lambda a: ctypes.c_void_p(a.ctypes.data)
outs = [pairs.copy(), pairs.copy()]
if threads:
    for k in (0, 1):                     # first call of each library starts its pool
        os.environ["BSW_HOST_THREADS"] = threads[k]
        assert libs[k].bsw_get_scores(ctxs[k], P(outs[k]), P(ref), P(qer), len(pairs), 100, 16) == 0
    print("host threads:", threads)
ts = [[], []]
for r in range(reps + 1):
    for k in (0, 1) if r % 2 == 0 else (1, 0):
        buf = outs[k]
        t = time.perf_counter()
        assert libs[k].bsw_get_scores(ctxs[k], P(buf), P(ref), P(qer), len(buf), 100, 16) == 0
        if r > 0:
            ts[k].append(time.perf_counter() - t)
same = all(np.array_equal(outs[0][f], outs[1][f]) for f in bsw.OUT_FIELDS)
for k in (0, 1):
    v = sorted(ts[k])
    print(f"{os.path.basename(sys.argv[1 + k])}: median {statistics.median(v)*1e3:.2f} ms = "
          f"{len(pairs)/statistics.median(v)/1e6:.1f} M/s, best {v[0]*1e3:.2f} ms, q25 {v[len(v)//4]*1e3:.2f} ms")
print("outputs identical:", same)
