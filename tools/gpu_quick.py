"""First GPU check: parity of the HIP path vs the CPU oracle + rough timing (dev tool)."""
import sys, os, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'bwa-mem2-arm_amd', 'py')]
import oracle, bswgen, bsw

P = oracle.make_params()
os.environ['BSW_PK'] = '1'          # exercise the packed kernel for its eligible pairs
eng = bsw.Engine()
os.environ.pop('BSW_PK')
def check(name, pairs, ref, qer, w):
    a = pairs.copy(); b = pairs.copy()
    oracle.get_scores(P, a, ref, qer, w, nthreads=16)
    t = time.time(); eng.get_scores(b, ref, qer, w); dt = time.time() - t
    bad = np.zeros(len(a), bool)
    for f in bsw.OUT_FIELDS:
        bad |= a[f] != b[f]
    st = eng.last_stats()
    print(f"{name:24s} n={len(a):8d} w={w:4d} mismatches={int(bad.sum()):6d}  call {dt*1e3:8.2f} ms  kernel {st.kernel_ms:8.3f} ms  i16={st.n_i16} wide={st.n_wide} launches={st.n_launches}", flush=True)
    if bad.any():
        k = np.flatnonzero(bad)[:5]
        for i in k:
            print('   idx', i, 'len', a[i]['len1'], a[i]['len2'], 'h0', a[i]['h0'], 'oracle', [int(a[i][f]) for f in bsw.OUT_FIELDS], 'gpu', [int(b[i][f]) for f in bsw.OUT_FIELDS])
    return int(bad.sum())

tot = 0
tot += check('edge', *bswgen.edge_pairs(), 100)
for w in (1, 5, 100):
    tot += check('random', *bswgen.random_pairs(4000, seed=w), w)
tot += check('random-long', *bswgen.random_pairs(500, seed=9, qlen=(150, 400), tlen=(100, 500)), 100)
tot += check('c2-like', *bswgen.c2_like(20000, seed=3), 100)
# packed-kernel class: qlen 129..160, h0 + min(qlen, tlen) <= 255
for w in (0, 1, 7, 40, 100, 200):
    tot += check('pk-random', *bswgen.random_pairs(6000, seed=70 + w, qlen=(129, 160), tlen=(0, 330), h0=(0, 95)), w)
tot += check('pk-random-h0hi', *bswgen.random_pairs(6000, seed=5, qlen=(129, 160), tlen=(0, 330), h0=(0, 140)), 100)
p, r, q = bsw.synth_batch(1000000)
check('synth-c2 1M', p, r, q, 100)
for _ in range(2):
    b = p.copy(); t = time.time(); eng.get_scores(b, r, q, 100); dt = time.time() - t
    st = eng.last_stats()
    print(f"synth 1M: call {dt*1e3:.1f} ms kernel {st.kernel_ms:.3f} ms -> {1e6/(st.kernel_ms*1e-3)/1e6:.1f} M pairs/s (kernel)")
eng2 = bsw.Engine()                 # default routing: lane kernel
for _ in range(2):
    b = p.copy(); eng2.get_scores(b, r, q, 100)
    st = eng2.last_stats()
    print(f"synth 1M lane kernel (default): kernel {st.kernel_ms:.3f} ms -> {1e6/(st.kernel_ms*1e-3)/1e6:.1f} M pairs/s")
print('TOTAL MISMATCHES', tot)
