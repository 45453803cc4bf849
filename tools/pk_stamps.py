"""Per-row-phase cycle split of the packed kernel (diagnostic build with -DBSW_PK_STAMPS; dev tool).
usage: python tools/pk_stamps.py exp/libbsw_pk_stamps.so"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'bwa-mem2-arm_amd', 'py'))
import hiprt, bsw
pairs, ref, qer = bsw.synth_batch(1_000_000)
L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
P = ctypes.c_void_p
L.bsw_create.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(P)]
L.bsw_get_scores_device.argtypes = [P, P, P, P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int, P]
L.bsw_last_stats.argtypes = [P, P]
ctx = P(); prm = bsw.default_params()
assert L.bsw_create(ctypes.byref(prm), 0, 1, ctypes.byref(ctx)) == 0
for rnd in range(2):
    dp = hiprt.DeviceBuffer.from_array(pairs); dr = hiprt.DeviceBuffer.from_array(ref); dq = hiprt.DeviceBuffer.from_array(qer)
    assert L.bsw_get_scores_device(ctx, P(dp.ptr), P(dr.ptr), P(dq.ptr), len(pairs), 100, 16, None) == 0
    st = bsw.Stats(); L.bsw_last_stats(ctx, ctypes.byref(st))
    got = dp.download(np.empty_like(pairs))
# A-halves carry acc0/acc1/acc4 in seqid/regid/id, B-halves acc2/acc3: a lane's A and B are
# different pairs, so average over all pairs that carry each field.
a0 = got['seqid'].astype(np.uint32).astype(np.float64)
a1 = got['regid'].astype(np.uint32).astype(np.float64)
idf = got['id'].astype(np.uint32).astype(np.float64)
isA = idf != pairs['id'].astype(np.uint32)   # A halves overwrote id
print('kernel ms', st.kernel_ms, 'A halves', int(isA.sum()))
names = ['bounds+reduce', 'target+setup', 'groups', 'row-end', 'loop tail']
vals = [a0[isA].mean(), a1[isA].mean(), a0[~isA].mean(), a1[~isA].mean(), idf[isA].mean()]
tot = sum(vals)
for n, v in zip(names, vals):
    print(f'{n:16s} {v/1e3:10.1f} K cycles/wave  {100*v/tot:5.1f}%')
print(f'{"total":16s} {tot/1e3:10.1f} K cycles/wave')
