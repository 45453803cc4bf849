"""Byte-wide H/E planes (BSW_OPT_KERNEL8 = 2): the packed-column kernel with the 8-bit regime's
cells stored as bytes (bsw_pc.hip, pcb_group) -- half the plane registers, three waves per SIMD
at QMAX 160 instead of two.  Integer path: outputs must equal the CPU oracle (ksw_extend2)
bit for bit on every pair, with the same routing as the int16-plane form (pairs outside the
8-bit regime fall back to the int16 lane kernel: BASELINE configs[2]'s overflow fallback)."""

import numpy as np
import pytest

import bsw
import bswgen
import hiprt
import oracle
from ksw_ext_ref import bwa_fill_scmat

pytestmark = pytest.mark.gpu


def _oparams(sc=None):
    if sc is None:
        return oracle.make_params()
    return oracle.make_params(o_del=sc["o_del"], e_del=sc["e_del"], o_ins=sc["o_ins"],
                              e_ins=sc["e_ins"], zdrop=sc["zdrop"], end_bonus=sc["end_bonus"],
                              mat=bwa_fill_scmat(sc["a"], sc["b"]))


def _gparams(sc=None):
    if sc is None:
        return bsw.default_params()
    return bsw.default_params(a=sc["a"], b=sc["b"], o_del=sc["o_del"], e_del=sc["e_del"],
                              o_ins=sc["o_ins"], e_ins=sc["e_ins"], zdrop=sc["zdrop"],
                              end_bonus=sc["end_bonus"])


def _assert_same(want, got, tag=""):
    bad = np.zeros(len(want), bool)
    for f in bsw.OUT_FIELDS:
        bad |= want[f] != got[f]
    if bad.any():
        i = int(np.flatnonzero(bad)[0])
        raise AssertionError(f"{tag}: {int(bad.sum())} of {len(want)} pairs differ; first idx {i} "
                             f"len1={want[i]['len1']} len2={want[i]['len2']} h0={want[i]['h0']} "
                             f"want={[int(want[i][f]) for f in bsw.OUT_FIELDS]} "
                             f"got={[int(got[i][f]) for f in bsw.OUT_FIELDS]}")


@pytest.fixture(scope="module")
def eng8():
    e = bsw.Engine(kernel8=2, small_batch=0, mid_batch=0)   # planned path: the pc classes
    yield e
    e.close()


@pytest.mark.parametrize("cell_bits", [16, 8])
def test_byte_planes_golden(golden, cell_bits):
    engines = {}
    for name, pairs, ref, qer, w, sc in golden:
        key = tuple(sorted(sc.items()))
        if key not in engines:
            engines[key] = bsw.Engine(_gparams(sc), kernel8=2, small_batch=0, mid_batch=0)
        got = pairs.copy()
        for f in bsw.OUT_FIELDS:
            got[f] = -9
        engines[key].get_scores(got, ref, qer, w, cell_bits)
        _assert_same(pairs, got, f"byte planes golden {name} cb={cell_bits}")


@pytest.mark.parametrize("w", [0, 1, 7, 40, 100, 200])
def test_byte_planes_random(eng8, w):
    pairs, ref, qer = bswgen.random_pairs(6000, seed=370 + w, qlen=(0, 159), tlen=(0, 330), h0=(0, 95))
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
    eng8.get_scores(got, ref, qer, w)
    _assert_same(want, got, f"byte planes w={w}")
    assert eng8.last_stats().n_packed == len(pairs)


def test_byte_planes_bucket_edges_and_bound(eng8):
    """qlen at every QMAX bucket edge, h0 exactly at the 8-bit bound (H reaches 255: the byte's
    top value) and one above it (int16 fallback)."""
    rng = np.random.default_rng(21)
    shapes = []
    for q in (0, 1, 2, 3, 4, 5, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 159, 160, 161):
        for t in (0, 1, 3, q, q + 1, 2 * q + 7, 300):
            shapes.append((t, q, int(min(rng.integers(0, 120), max(0, 255 - min(q, t))))))
            shapes.append((t, q, max(0, 255 - min(q, t))))
            shapes.append((t, q, 256 - min(q, t)))
    pairs, ref, qer = bswgen.pairs_from_shapes(shapes, seed=22)
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    eng8.get_scores(got, ref, qer, 100, cell_bits=8)
    _assert_same(want, got, "byte planes bucket edges")
    assert eng8.last_stats().n_packed > 0


def test_byte_planes_score_255():
    """Identical query and target with h0 = 255 - qlen: every diagonal cell climbs to exactly
    255 (the byte's top value) -- stored, unpacked and keyed without wrapping."""
    for q in (20, 64, 100, 150, 158):
        rng = np.random.default_rng(q)
        seq = rng.integers(0, 4, q, dtype=np.uint8)
        shapes = [(q, q, 255 - q)] * 64
        pairs, ref, qer = bswgen.pairs_from_shapes(shapes, seed=q)
        for k in range(len(pairs)):
            ref[pairs[k]["idr"]:pairs[k]["idr"] + q] = seq
            qer[pairs[k]["idq"]:pairs[k]["idq"] + q] = seq
        want, got = pairs.copy(), pairs.copy()
        oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=4)
        assert int(want["score"].max()) == 255
        e = bsw.Engine(kernel8=2, small_batch=0, mid_batch=0)
        e.get_scores(got, ref, qer, 100, cell_bits=8)
        _assert_same(want, got, f"score 255 q={q}")
        assert e.last_stats().n_packed == len(pairs)
        e.close()


@pytest.mark.parametrize("q", [4, 5, 7, 64, 97, 149, 150, 151, 158])
def test_byte_planes_qlen_tail(eng8, q):
    cfg = bsw.synth_cfg(qlen=q, tlen=2 * q + 3, h0_lo=0, h0_hi=min(95, 255 - q))
    pairs, ref, qer = bsw.synth_batch(8192, pair_base=7000 * q, cfg=cfg)
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    eng8.get_scores(got, ref, qer, 100)
    _assert_same(want, got, f"byte planes qlen tail q={q}")


def test_byte_planes_c3_fallback(eng8):
    """C3 (BASELINE configs[2]) shape: h0 up to 130, so ~22% of the pairs leave the 8-bit
    regime for the int16 lane kernel; the rest run on byte cells.  200K pairs vs the oracle."""
    cfg = bsw.synth_cfg(h0_hi=130)
    pairs, ref, qer = bsw.synth_batch(200_000, pair_base=11, cfg=cfg)
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=16)
    dp = hiprt.DeviceBuffer.from_array(pairs)
    dr = hiprt.DeviceBuffer.from_array(ref)
    dq = hiprt.DeviceBuffer.from_array(qer)
    eng8.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), 100, 8)
    got = dp.download(np.empty_like(pairs))
    _assert_same(want, got, "byte planes C3")
    st = eng8.last_stats()
    assert st.n_u8 == st.n_packed and 0 < st.n_i16 < len(pairs) // 2
    assert st.n_u8 + st.n_i16 + st.n_wide == len(pairs)


def test_byte_planes_c2_sample_device(eng8):
    pairs, ref, qer = bsw.synth_batch(300_000)
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=16)
    dp = hiprt.DeviceBuffer.from_array(pairs)
    dr = hiprt.DeviceBuffer.from_array(ref)
    dq = hiprt.DeviceBuffer.from_array(qer)
    eng8.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), 100)
    got = dp.download(np.empty_like(pairs))
    _assert_same(want, got, "byte planes C2 300K")
    assert eng8.last_stats().n_packed == len(pairs)
