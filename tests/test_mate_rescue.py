"""Mate-rescue batch (include/bsw_mate.h): upstream ksw_align2 /
ksw_u8 / ksw_i16 semantics.

CPU tests pin the oracle (oracle/ksw_align_ref.c, a literal striped restatement of the SSE2
kernels) against an independent non-striped formulation (tests/ksw_align_py.py) -- the
formulation the GPU kernel implements -- on random inputs covering u8 / i16, every KSW_X*
flag combination, asymmetric gaps, other match / mismatch scores, N bases, empty and
one-base sequences and the u8 saturation stop.  GPU tests require bsw_ksw_align2 to equal
the oracle job for job.  Parity is unpinned by the reference (no ksw sources or fixtures
ship in /root/reference)."""

import random

import numpy as np
import pytest

import bsw
import oracle
import ksw_align_py as kp
from ksw_ext_ref import bwa_fill_scmat

XS = (0, kp.KSW_XBYTE, kp.KSW_XSTART, kp.KSW_XSTART | kp.KSW_XBYTE, kp.KSW_XSUBO | 5,
      kp.KSW_XSUBO | kp.KSW_XSTART | 19, kp.KSW_XSUBO | kp.KSW_XSTART | kp.KSW_XBYTE | 19,
      kp.KSW_XSUBO | kp.KSW_XSTART | kp.KSW_XBYTE | 0, kp.KSW_XSTOP | 30)


def _case(rnd, qmax=90, tmax=140):
    qlen, tlen = rnd.randint(0, qmax), rnd.randint(0, tmax)
    if qlen and tlen >= qlen and rnd.random() < 0.7:            # query planted with edits
        tg = [rnd.randrange(4) for _ in range(tlen)]
        k = rnd.randint(0, tlen - qlen)
        q = []
        while len(q) < qlen:
            r = rnd.random()
            if r < 0.04:
                q.append(rnd.randrange(5))
            elif r < 0.07:
                k += rnd.randint(1, 4)
            elif r < 0.10:
                q += [rnd.randrange(4) for _ in range(rnd.randint(1, 4))]
            else:
                q.append(tg[k] if k < tlen else rnd.randrange(4))
                k += 1
        q = q[:qlen]
    else:
        q = [rnd.randrange(5) for _ in range(qlen)]
        tg = [rnd.randrange(5) for _ in range(tlen)]
    return q, tg


@pytest.mark.parametrize("seed", range(4))
def test_oracle_striped_equals_query_order_formulation(seed):
    rnd = random.Random(100 + seed)
    for _ in range(150):
        q, tg = _case(rnd)
        a, b = rnd.choice([(1, 4), (1, 3), (2, 5), (1, 1)])
        mat = bwa_fill_scmat(a, b)
        od, ed, oi, ei = rnd.randint(0, 8), rnd.randint(1, 3), rnd.randint(1, 8), rnd.randint(1, 3)
        xtra = rnd.choice(XS)
        want = oracle.ksw_align2(q, tg, mat, od, ed, oi, ei, xtra)
        got = kp.ksw_align2(q, tg, mat, od, ed, oi, ei, xtra)
        assert want == got, (len(q), len(tg), hex(xtra), (od, ed, oi, ei), a, b, want, got)


def test_u8_saturation_stop():
    """ksw_u8 stops once gmax + shift >= 255 and reports 255 without qe / score2; ksw_i16
    reports the true score."""
    rnd = random.Random(7)
    q = [rnd.randrange(4) for _ in range(256)]
    tg = [rnd.randrange(4) for _ in range(20)] + q + [rnd.randrange(4) for _ in range(20)]
    mat = bwa_fill_scmat()
    x = kp.KSW_XSUBO | kp.KSW_XSTART | 19
    r8 = oracle.ksw_align2(q, tg, mat, 6, 1, 6, 1, x | kp.KSW_XBYTE)
    assert r8 == kp.ksw_align2(q, tg, mat, 6, 1, 6, 1, x | kp.KSW_XBYTE)
    assert r8[0] == 255 and r8[2] == -1 and r8[3] == -1 and r8[5] == -1
    r16 = oracle.ksw_align2(q, tg, mat, 6, 1, 6, 1, x)
    assert r16 == kp.ksw_align2(q, tg, mat, 6, 1, 6, 1, x)
    assert r16[:3] == [256, 20 + 255, 255] and r16[5:] == [20, 0]


def test_secondary_hit_and_start():
    """Two copies of the query: score2 / te2 find the second outside the exclusion window;
    tb / qb the start of the first."""
    rnd = random.Random(9)
    q = [rnd.randrange(4) for _ in range(60)]
    gap = [rnd.randrange(4) for _ in range(100)]
    tg = gap[:10] + q + gap + q[:50] + gap[:5]
    mat = bwa_fill_scmat()
    x = kp.KSW_XSUBO | kp.KSW_XSTART | kp.KSW_XBYTE | 19
    r = oracle.ksw_align2(q, tg, mat, 6, 1, 6, 1, x)
    assert r == kp.ksw_align2(q, tg, mat, 6, 1, 6, 1, x)
    assert r[0] == 60 and r[1] == 69 and r[2] == 59 and r[5:] == [10, 0]
    assert r[3] == 50 and r[4] == 10 + 60 + 100 + 49


def test_mate_generator_shape():
    ref = bsw.synth_reference(300_000, seed=3)
    pairs, qer = bsw.synth_mates(ref, 400, cfg=bsw.mates_cfg(seed=2))
    assert np.all(pairs["len1"] == 550) and np.all(pairs["len2"] == 150)
    assert np.all(pairs["h0"] == (kp.KSW_XSUBO | kp.KSW_XSTART | kp.KSW_XBYTE | 19))
    out = oracle.ksw_align2_batch(pairs, ref, qer, bwa_fill_scmat(), nthreads=8)
    good = out["score"] >= 50                          # windows holding the mate
    assert 0.7 < good.mean() < 0.9
    assert np.all(out["tb"][good] >= 0) and np.all(out["qb"][good] >= 0)
    assert np.all(out["score"][~good] < 30)


# ---------------------------------------------------------------- GPU: engine == oracle
def _random_batch(n, seed, qmax=256, tmax=700):
    rnd = random.Random(seed)
    pairs = np.zeros(n, dtype=bsw.SEQPAIR_DTYPE)
    refs, qers, ro, qo = [], [], 0, 0
    for i in range(n):
        q, tg = _case(rnd, qmax, tmax)
        pairs[i]["idr"], pairs[i]["idq"], pairs[i]["len1"], pairs[i]["len2"] = ro, qo, len(tg), len(q)
        pairs[i]["h0"] = rnd.choice(XS)
        pairs[i]["id"] = i
        refs.append(tg)
        qers.append(q)
        ro += len(tg)
        qo += len(q)
    ref = np.array([b for t in refs for b in t] + [0], dtype=np.uint8)
    qer = np.array([b for t in qers for b in t] + [0], dtype=np.uint8)
    return pairs, ref, qer


def _same(want, got, tag):
    bad = np.zeros(len(want), bool)
    for f in bsw.KSWR_DTYPE.names:
        bad |= want[f] != got[f]
    if bad.any():
        i = int(np.flatnonzero(bad)[0])
        raise AssertionError(f"{tag}: {int(bad.sum())}/{len(want)} jobs differ; first {i}: want {want[i]} "
                             f"got {got[i]}")


@pytest.mark.gpu
@pytest.mark.parametrize("scoring", [(1, 4, 6, 1, 6, 1), (1, 3, 5, 2, 3, 1), (2, 5, 0, 1, 1, 2)])
def test_gpu_random_jobs_match_oracle(scoring):
    a, b, od, ed, oi, ei = scoring
    pairs, ref, qer = _random_batch(3000, seed=a * 100 + od)
    p = bsw.default_params(a=a, b=b, o_del=od, e_del=ed, o_ins=oi, e_ins=ei)
    want = oracle.ksw_align2_batch(pairs, ref, qer, list(p.mat), od, ed, oi, ei, nthreads=16)
    eng = bsw.Engine(p)
    got = bsw.ksw_align2(eng, pairs, ref, qer)
    _same(want, got, f"random jobs {scoring}")
    st = bsw.mate_last_stats(eng)
    assert st.n_fwd == len(pairs) and st.n_rev > 0 and st.cells_fwd > 0
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("read_len,win_len,xbyte", [(150, 550, True), (150, 550, False), (101, 400, True),
                                                    (250, 700, False)])
def test_gpu_mate_jobs_match_oracle(read_len, win_len, xbyte):
    ref = bsw.synth_reference(4_000_000, seed=11)
    pairs, qer = bsw.synth_mates(ref, 20_000, cfg=bsw.mates_cfg(seed=read_len, read_len=read_len,
                                                                 win_len=win_len))
    if not xbyte:
        pairs["h0"] &= ~kp.KSW_XBYTE
    want = oracle.ksw_align2_batch(pairs, ref, qer, bwa_fill_scmat(), nthreads=16)
    eng = bsw.Engine()
    got = bsw.ksw_align2(eng, pairs, ref, qer)
    _same(want, got, f"mate jobs {read_len}/{win_len} xbyte={xbyte}")
    eng.close()


@pytest.mark.gpu
def test_gpu_edges():
    """Empty query / target, one base, all-N, u8 saturation, query at the 256 limit."""
    rnd = random.Random(3)
    jobs = [([], [1, 2]), ([1], []), ([], []), ([2], [2]), ([4] * 30, [4] * 50),
            ([rnd.randrange(4) for _ in range(256)], None), ([0, 1, 2, 3] * 40, [0, 1, 2, 3] * 100)]
    pairs = np.zeros(len(jobs) * len(XS), dtype=bsw.SEQPAIR_DTYPE)
    refb, qerb = [], []
    k = 0
    for q, tg in jobs:
        if tg is None:
            tg = [rnd.randrange(4) for _ in range(9)] + q + [rnd.randrange(4) for _ in range(9)]
        for x in XS:
            pairs[k]["idr"], pairs[k]["idq"] = len(refb), len(qerb)
            pairs[k]["len1"], pairs[k]["len2"], pairs[k]["h0"] = len(tg), len(q), x
            refb += tg
            qerb += q
            k += 1
    ref = np.array(refb + [0], dtype=np.uint8)
    qer = np.array(qerb + [0], dtype=np.uint8)
    want = oracle.ksw_align2_batch(pairs, ref, qer, bwa_fill_scmat())
    eng = bsw.Engine()
    got = bsw.ksw_align2(eng, pairs, ref, qer)
    _same(want, got, "edges")
    eng.close()


@pytest.mark.gpu
def test_gpu_rejects_unsupported():
    eng = bsw.Engine(bsw.default_params(o_ins=0))
    pairs, ref, qer = _random_batch(10, seed=1, qmax=20, tmax=30)
    with pytest.raises(bsw.BswError):
        bsw.ksw_align2(eng, pairs, ref, qer)
    eng.close()
    eng = bsw.Engine()
    pairs["len2"][3] = 300                                      # > BSW_MATE_MAX_QLEN
    with pytest.raises(bsw.BswError):
        bsw.ksw_align2(eng, pairs, np.zeros(10_000, np.uint8), np.zeros(10_000, np.uint8))
    eng.close()


@pytest.mark.gpu
def test_gpu_all_devices_context():
    """A context over every visible device shards host-buffer calls by contiguous job ranges."""
    import hiprt
    ref = bsw.synth_reference(2_000_000, seed=19)
    pairs, qer = bsw.synth_mates(ref, 9_000)
    want = oracle.ksw_align2_batch(pairs, ref, qer, bwa_fill_scmat(), nthreads=16)
    eng = bsw.Engine(n_gpus=hiprt.device_count())
    got = bsw.ksw_align2(eng, pairs, ref, qer)
    _same(want, got, f"n_gpus={hiprt.device_count()}")
    assert bsw.mate_last_stats(eng).n_fwd == len(pairs)
    eng.close()
