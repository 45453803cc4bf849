"""Global alignment with traceback (include/bsw_global.h): upstream
ksw_global2 semantics, as bwa_gen_cigar2 calls it for every final alignment.

CPU tests pin the oracle (oracle/ksw_global_ref.c, a literal restatement of the single-row
eh[] code) against an independent band-matrix formulation (tests/ksw_global_py.py) on random
inputs -- asymmetric gaps, other match / mismatch scores, N bases, empty and one-base
sequences, bands narrower and wider than the query -- plus hand-derived known answers and two
properties of every traced CIGAR: it spans exactly qlen query and tlen target bases, and
re-scoring it with affine gaps gives the returned score.  GPU tests require
bsw_ksw_global2 to equal the oracle job for job (score, CIGAR, op count).  Parity is unpinned
by the reference (no ksw sources or fixtures ship in /root/reference)."""

import random

import numpy as np
import pytest

import bsw
import oracle
import ksw_global_py as kg
from ksw_ext_ref import bwa_fill_scmat


def _case(rnd, qmax=60, tmax=70):
    """(query, target, w) with the traceback start inside the band (qlen >= tlen - w)."""
    if rnd.random() < 0.6:                       # related: target = query with edits
        q = [rnd.randrange(4) for _ in range(rnd.randint(1, qmax))]
        t = []
        for b in q:
            r = rnd.random()
            if r < 0.05:
                t.append(rnd.randrange(5))
            elif r < 0.08:
                continue
            elif r < 0.11:
                t += [b] + [rnd.randrange(4) for _ in range(rnd.randint(1, 3))]
            else:
                t.append(b)
        t = t[:tmax]
    else:
        q = [rnd.randrange(5) for _ in range(rnd.randint(0, qmax))]
        t = [rnd.randrange(5) for _ in range(rnd.randint(0, tmax))]
    w = rnd.choice([0, 1, 2, 5, 10, 35, 100])
    if q and t and len(q) < len(t) - w:
        w = len(t) - len(q) + rnd.randint(0, 3)
    return q, t, w


@pytest.mark.parametrize("seed", range(4))
def test_oracle_equals_band_matrix_formulation(seed):
    rnd = random.Random(500 + seed)
    for _ in range(120):
        q, t, w = _case(rnd)
        a, b = rnd.choice([(1, 4), (1, 3), (2, 5), (1, 1)])
        mat = bwa_fill_scmat(a, b)
        od, ed, oi, ei = rnd.randint(0, 8), rnd.randint(1, 3), rnd.randint(0, 8), rnd.randint(1, 3)
        want = oracle.ksw_global2(q, t, mat, od, ed, oi, ei, w)
        got = kg.ksw_global2(q, t, mat, od, ed, oi, ei, w)
        assert want == got, (len(q), len(t), w, (od, ed, oi, ei), a, b, want, got)


@pytest.mark.parametrize("seed", range(3))
def test_traced_cigar_spans_and_rescores(seed):
    """Every CIGAR spans qlen / tlen and scores (affine, one open per run) to the DP score."""
    rnd = random.Random(900 + seed)
    for _ in range(200):
        q, t, w = _case(rnd)
        a, b = rnd.choice([(1, 4), (2, 5)])
        mat = bwa_fill_scmat(a, b)
        od, ed, oi, ei = rnd.randint(1, 8), rnd.randint(1, 3), rnd.randint(1, 8), rnd.randint(1, 3)
        sc, cig = oracle.ksw_global2(q, t, mat, od, ed, oi, ei, w)
        if sc <= kg.NEG // 2:                         # last column never reached: no path
            continue
        rs, ti, qj = kg.rescore(q, t, mat, od, ed, oi, ei, cig)
        assert (ti, qj) == (len(t), len(q)), (cig, len(t), len(q))
        assert rs == sc, (q, t, w, cig, sc, rs)


def test_known_answers():
    mat = bwa_fill_scmat()
    # K1: identical sequences -> L*a, one M run
    q = [0, 1, 2, 3, 0, 1, 2]
    assert oracle.ksw_global2(q, q, mat, 6, 1, 6, 1, 5) == (7, [(0, 7)])
    # K2: empty query -> deletion of the whole target, -(o_del + e_del * tlen)
    assert oracle.ksw_global2([], [0, 1, 2], mat, 6, 1, 6, 1, 5) == (-9, [(2, 3)])
    # K3: empty target -> insertion of the query (qlen <= w): -(o_ins + e_ins * qlen)
    assert oracle.ksw_global2([0, 1], [], mat, 6, 1, 6, 1, 5) == (-8, [(1, 2)])
    # K4: one extra target base (a doubled 2): 6 matches - (6 + 1) = -1.  Walking back the
    # traceback prefers M (d = 0 on ties), so the deletion lands on the LEFT copy: 2M 1D 4M
    assert oracle.ksw_global2([0, 1, 2, 3, 0, 1], [0, 1, 2, 2, 3, 0, 1], mat, 6, 1, 6, 1, 5) == \
        (-1, [(0, 2), (2, 1), (0, 4)])
    # K5: a single mismatch beats an insertion + deletion: 3 - 4 = -1, all M
    assert oracle.ksw_global2([0, 1, 2, 3], [0, 1, 3, 3], mat, 6, 1, 6, 1, 5) == (-1, [(0, 4)])
    # K6: both empty -> 0, no ops
    assert oracle.ksw_global2([], [], mat, 6, 1, 6, 1, 5) == (0, [])


def test_gen_cigar_band_rule():
    """bwa_gen_cigar2's w for 150 bp reads under bwa defaults: (70 + |d| + 1) >> 1, >= |d| + 3."""
    assert kg.gen_cigar_w(150, 150, 100, 1, 6, 1, 6, 1) == 35
    assert kg.gen_cigar_w(150, 153, 100, 1, 6, 1, 6, 1) == 37
    assert kg.gen_cigar_w(150, 150, 10, 1, 6, 1, 6, 1) == 10
    assert kg.gen_cigar_w(10, 40, 100, 1, 6, 1, 6, 1) == 33


def test_oracle_batch_flags():
    """Batch form: -2 for the undefined geometry, -1 on CIGAR overflow, scores always."""
    mat = bwa_fill_scmat()
    rnd = random.Random(3)
    q = [rnd.randrange(4) for _ in range(40)]
    t = q[:10] + [rnd.randrange(4) for _ in range(60)]
    pairs = np.zeros(3, dtype=oracle.SEQPAIR_DTYPE)
    ref = np.array(t + q, dtype=np.uint8)
    qer = np.array(q, dtype=np.uint8)
    pairs[0] = (0, 0, 0, 70, 40, 5, 0, 0, 0, 0, 0, 0, 0, 0)      # 40 < 70 - 5: undefined -> -2
    pairs[1] = (70, 0, 1, 40, 40, 5, 0, 0, 0, 0, 0, 0, 0, 0)     # identical -> 40M
    pairs[2] = (0, 0, 2, 70, 40, 40, 0, 0, 0, 0, 0, 0, 0, 0)     # many ops, stride 2 -> -1
    sc, cig, nc = oracle.ksw_global2_batch(pairs, ref, qer, mat, stride=2)
    assert nc[0] == -2 and nc[1] == 1 and cig[1, 0] == (40 << 4) and sc[1] == 40 and nc[2] == -1
    sc2, _, _ = oracle.ksw_global2_batch(pairs, ref, qer, mat, stride=0)
    assert np.array_equal(sc, sc2)


def test_global_generator_shape():
    ref = bsw.synth_reference(2_000_000, seed=5)
    pairs, qer = bsw.synth_globals(ref, 500)
    assert np.all(pairs["len2"] == 150)
    d = pairs["len1"] - pairs["len2"]
    assert np.all(np.abs(d) <= 20)
    w = np.array([kg.gen_cigar_w(150, int(l1), 100, 1, 6, 1, 6, 1) for l1 in pairs["len1"]])
    assert np.array_equal(pairs["h0"], w)
    sc, cig, nc = oracle.ksw_global2_batch(pairs, ref, qer, bwa_fill_scmat(), stride=64, nthreads=8)
    assert np.all(nc > 0) and np.median(sc) > 120


# ---------------------------------------------------------------- GPU: engine == oracle
def _random_batch(n, seed, qmax=60, tmax=70):
    rnd = random.Random(seed)
    pairs = np.zeros(n, dtype=bsw.SEQPAIR_DTYPE)
    refs, qers, ro, qo = [], [], 0, 0
    for i in range(n):
        q, tg, w = _case(rnd, qmax, tmax)
        pairs[i]["idr"], pairs[i]["idq"], pairs[i]["len1"], pairs[i]["len2"] = ro, qo, len(tg), len(q)
        pairs[i]["h0"] = w
        pairs[i]["id"] = i
        refs.append(tg)
        qers.append(q)
        ro += len(tg)
        qo += len(q)
    ref = np.array([b for t in refs for b in t] + [0], dtype=np.uint8)
    qer = np.array([b for t in qers for b in t] + [0], dtype=np.uint8)
    return pairs, ref, qer


def _check(want, got, tag):
    ws, wc, wn = want
    gs, gc, gn = got
    bad = (ws != gs) | (wn != gn)
    if wc is not None:
        for i in np.flatnonzero(~bad):
            k = wn[i]
            if k > 0 and not np.array_equal(wc[i, :k], gc[i, :k]):
                bad[i] = True
    if bad.any():
        i = int(np.flatnonzero(bad)[0])
        k = max(int(wn[i]), 0)
        raise AssertionError(f"{tag}: {int(bad.sum())}/{len(ws)} jobs differ; first {i}: want "
                             f"{ws[i]} {wn[i]} {wc[i, :k] if wc is not None else ''} got {gs[i]} {gn[i]} "
                             f"{gc[i, :k] if gc is not None else ''}")


@pytest.fixture(params=["column", "band"])
def routing(request):
    """Default routing (column kernel first) or BSW_OPT_GLOB_BAND = 1 (band kernel first), set on
    every engine the test creates (through _engine)."""
    return request.param


def _engine(params, routing):
    return bsw.Engine(params, glob_band=1 if routing == "band" else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("scoring", [(1, 4, 6, 1, 6, 1), (1, 3, 5, 2, 3, 1), (2, 5, 0, 1, 1, 2)])
def test_gpu_random_jobs_match_oracle(scoring, routing):
    a, b, od, ed, oi, ei = scoring
    pairs, ref, qer = _random_batch(4000, seed=a * 100 + od + b)
    p = bsw.default_params(a=a, b=b, o_del=od, e_del=ed, o_ins=oi, e_ins=ei)
    want = oracle.ksw_global2_batch(pairs, ref, qer, list(p.mat), od, ed, oi, ei, stride=96, nthreads=16)
    eng = _engine(p, routing)
    got = bsw.ksw_global2(eng, pairs, ref, qer, stride=96)
    _check(want, got, f"random jobs {scoring}")
    assert np.array_equal(pairs["score"], want[0])
    if routing == "column":
        # unrelated random pairs: many paths leave the column kernel's narrow traceback corridor and
        # take the full-window rerun -- both paths exercised, outputs equal the oracle above
        assert bsw.global_last_stats(eng).n_tb_retry > 0
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("read_len", [150, 101, 250])
def test_gpu_bwa_shaped_jobs_match_oracle(read_len, routing):
    ref = bsw.synth_reference(4_000_000, seed=13)
    pairs, qer = bsw.synth_globals(ref, 20_000, cfg=bsw.globals_cfg(seed=read_len, read_len=read_len))
    want = oracle.ksw_global2_batch(pairs, ref, qer, bwa_fill_scmat(), stride=64, nthreads=16)
    eng = _engine(None, routing)
    got = bsw.ksw_global2(eng, pairs, ref, qer, stride=64)
    _check(want, got, f"bwa-shaped {read_len}")
    st = bsw.global_last_stats(eng)
    assert st.n_jobs == len(pairs) and (st.n_wide > 0) == (read_len > 160)   # 250 bp: w ~ 60 -> wide
    assert st.n_lane + st.n_wide == len(pairs)
    if routing == "column" and read_len <= 160:
        # bwa-shaped jobs: the narrow corridor (3 dwords per row) serves nearly every traceback
        assert st.n_tb_retry < 0.05 * len(pairs), st.n_tb_retry
    eng.close()


@pytest.mark.gpu
def test_gpu_edges_and_flags(routing):
    """Empty sequences, w = 0, wide routing (qlen > 160 and int16-unsafe scores), the
    undefined geometry (-2), CIGAR overflow (-1) and the score-only mode."""
    rnd = random.Random(77)
    cases = [([], [], 3), ([], [1, 2, 3], 2), ([0, 1, 2], [], 5), ([0, 1, 2, 3, 0], [], 2),
             ([1], [1], 0), ([2] * 30, [2] * 33, 3), ([4] * 20, [4] * 20, 3),
             ([rnd.randrange(4) for _ in range(200)], [rnd.randrange(4) for _ in range(210)], 40),
             ([rnd.randrange(4) for _ in range(20)], [rnd.randrange(4) for _ in range(60)], 5)]
    pairs = np.zeros(len(cases), dtype=bsw.SEQPAIR_DTYPE)
    ro = qo = 0
    refs, qers = [], []
    for i, (q, t, w) in enumerate(cases):
        pairs[i]["idr"], pairs[i]["idq"], pairs[i]["len1"], pairs[i]["len2"], pairs[i]["h0"] = \
            ro, qo, len(t), len(q), w
        refs += t
        qers += q
        ro += len(t)
        qo += len(q)
    ref = np.array(refs + [0], dtype=np.uint8)
    qer = np.array(qers + [0], dtype=np.uint8)
    mat = bwa_fill_scmat()
    eng = _engine(None, routing)
    for stride in (512, 3):
        want = oracle.ksw_global2_batch(pairs, ref, qer, mat, stride=stride)
        got = bsw.ksw_global2(eng, pairs.copy(), ref, qer, stride=stride)
        _check(want, got, f"edges stride {stride}")
    assert want[2][-1] == -2
    s0 = bsw.ksw_global2(eng, pairs.copy(), ref, qer, stride=0)
    assert np.array_equal(s0[0], want[0])
    eng.close()
    # int16-unsafe scoring -> wide kernel
    p = bsw.default_params(a=40, b=60, o_del=100, e_del=30, o_ins=100, e_ins=30)
    pr, rf, qr = _random_batch(300, seed=5, qmax=150, tmax=160)
    want = oracle.ksw_global2_batch(pr, rf, qr, list(p.mat), 100, 30, 100, 30, stride=160)
    eng = _engine(p, routing)
    got = bsw.ksw_global2(eng, pr, rf, qr, stride=160)
    _check(want, got, "wide scoring")
    st = bsw.global_last_stats(eng)              # the larger jobs exceed the int16 bound
    assert st.n_lane > 0 and st.n_wide + st.n_lane == len(pr)
    assert st.n_wide > 0 or routing == "band"    # (band kernel: int32 cells, takes them when w is small)
    eng.close()


@pytest.mark.gpu
def test_gpu_all_devices_context():
    """A context over every visible device shards host-buffer calls by contiguous job ranges."""
    import hiprt
    ref = bsw.synth_reference(2_000_000, seed=17)
    pairs, qer = bsw.synth_globals(ref, 9_000)
    want = oracle.ksw_global2_batch(pairs, ref, qer, bwa_fill_scmat(), stride=64, nthreads=16)
    eng = bsw.Engine(n_gpus=hiprt.device_count())
    got = bsw.ksw_global2(eng, pairs, ref, qer, stride=64)
    _check(want, got, f"n_gpus={hiprt.device_count()}")
    assert bsw.global_last_stats(eng).n_jobs == len(pairs)
    eng.close()
