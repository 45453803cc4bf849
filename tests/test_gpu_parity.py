"""GPU parity tests: the HIP path, called through the C ABI (libbsw_hip.so), must produce
outputs bit-identical to the CPU oracle (ksw_extend2 semantics) -- score, tle, gtle, qle,
gscore, max_off for every pair.  Integer path: the tolerance is zero.

Coverage: committed golden fixtures (all scoring variants and band widths), mixed random
shapes incl. the wide (qlen > 160) kernel, the reference's planned partial-batch sizes,
edge cases, the full C2 workload (1M pairs, oracle on 16 host threads), size-independent
properties at full size (idempotence, permutation invariance, host API == device API),
concurrent callers, and argument errors."""

import threading

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
def eng():
    e = bsw.Engine(small_batch=0, mid_batch=0)   # kernel-class tests: small batches stay on their classes
    yield e
    e.close()


@pytest.mark.parametrize("cell_bits", [16, 8])
def test_golden_fixtures(golden, cell_bits):
    engines = {}
    for name, pairs, ref, qer, w, sc in golden:
        key = tuple(sorted(sc.items()))
        if key not in engines:
            engines[key] = bsw.Engine(_gparams(sc), small_batch=0, mid_batch=0)
        got = pairs.copy()
        for f in bsw.OUT_FIELDS:
            got[f] = -9
        engines[key].get_scores(got, ref, qer, w, cell_bits)
        _assert_same(pairs, got, f"golden {name} cell_bits={cell_bits}")


@pytest.mark.parametrize("w", [0, 1, 5, 10, 100, 200])
def test_random_mixed_shapes(eng, w):
    pairs, ref, qer = bswgen.random_pairs(3000, seed=500 + w, tlen=(0, 330), qlen=(0, 200))
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
    eng.get_scores(got, ref, qer, w)
    _assert_same(want, got, f"random w={w}")
    st = eng.last_stats()
    assert st.n_i16 + st.n_u8 + st.n_wide == len(pairs)


@pytest.mark.parametrize("no_fork", [False, True])
def test_class_launch_fork(eng, no_fork):
    """A batch spanning every kernel class (short/long queries up to the wide kernel) gives the
    oracle's results whether its class launches fork over the slot's side streams (default) or
    run serially on the caller's stream (BSW_OPT_FORK = 0, read per call)."""
    eng.set_option("fork", 0 if no_fork else 1)
    pairs, ref, qer = bswgen.random_pairs(4000, seed=77, tlen=(0, 700), qlen=(0, 400))
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    for _ in range(2):                                  # second call reuses the side streams
        got[:] = pairs
        eng.get_scores(got, ref, qer, 100)
        _assert_same(want, got, f"class launches no_fork={no_fork}")
    st = eng.last_stats()
    eng.set_option("fork", 1)
    assert st.n_launches >= 3 and st.n_wave > 0
    assert st.n_i16 + st.n_u8 + st.n_wide == len(pairs)


@pytest.mark.parametrize("route", [1, 0])
def test_long_queries(eng, route):
    """Queries past the register kernels' 160 columns: the wave-per-alignment kernel
    (BSW_OPT_LONG 1, default) or the int32 wide kernel (0) -- both equal the oracle."""
    eng.set_option("long", route)
    pairs, ref, qer = bswgen.random_pairs(300, seed=9, tlen=(100, 700), qlen=(161, 600))
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    eng.get_scores(got, ref, qer, 100)
    st = eng.last_stats()
    eng.set_option("long", 1)
    _assert_same(want, got, f"long queries route {route}")
    assert (st.n_wave if route else st.n_wide) == len(pairs)


@pytest.mark.parametrize("L", [250, 500, 1000])
def test_wave_kernel_long_reads(eng, L):
    """bwa-shaped extensions of L-bp reads (query = the target's prefix with substitutions and
    short indels, target window L + 100) on the wave kernel, w = 100 and the w << 1 retry band."""
    n = 400 if L < 1000 else 160
    pairs, ref, qer = bswgen.random_pairs(n, seed=L, tlen=(L + 50, L + 150), qlen=(L, L), h0=(1, 200),
                                          p_sub=(0.0, 0.05), p_indel=(0.0, 0.01))
    for w in (100, 200):
        want, got = pairs.copy(), pairs.copy()
        oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
        eng.get_scores(got, ref, qer, w)
        _assert_same(want, got, f"long reads L={L} w={w}")
        assert eng.last_stats().n_wave == n


def test_wave_kernel_forced_golden(golden):
    """Every golden batch whose scoring the wave kernel takes (max(mat) == 1), with every pair
    routed to it (BSW_OPT_LONG 2) -- short queries, empty sequences, w = 0 .. 200, z-drop off."""
    engines, ran = {}, 0
    for name, pairs, ref, qer, w, sc in golden:
        if sc.get("a", 1) != 1:
            continue
        key = tuple(sorted(sc.items()))
        if key not in engines:
            engines[key] = bsw.Engine(_gparams(sc), long=2)
        got = pairs.copy()
        for f in bsw.OUT_FIELDS:
            got[f] = -9
        engines[key].get_scores(got, ref, qer, w)
        _assert_same(pairs, got, f"golden {name} on the wave kernel")
        ran += engines[key].last_stats().n_wave
    assert ran > 0


@pytest.mark.parametrize("w", [0, 1, 7, 100, 200])
def test_wave_kernel_forced_random(w):
    e = bsw.Engine(long=2)
    pairs, ref, qer = bswgen.random_pairs(2000, seed=700 + w, tlen=(0, 400), qlen=(0, 300))
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
    e.get_scores(got, ref, qer, w)
    _assert_same(want, got, f"wave kernel random w={w}")
    assert e.last_stats().n_wave == len(pairs)
    e.close()


def test_edge_cases(eng):
    pairs, ref, qer = bswgen.edge_pairs(seed=3)
    for w in (0, 1, 100):
        want, got = pairs.copy(), pairs.copy()
        oracle.get_scores(_oparams(), want, ref, qer, w)
        eng.get_scores(got, ref, qer, w)
        _assert_same(want, got, f"edge w={w}")


@pytest.mark.parametrize("m", [1, 15, 31, 32, 33, 50, 63, 64, 65, 100, 255, 257])
def test_partial_batches(eng, m):
    pairs, ref, qer = bswgen.c2_like(m, seed=m)
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100)
    eng.get_scores(got, ref, qer, 100)
    _assert_same(want, got, f"partial {m}")


def test_nondefault_scoring_generic_kernel():
    sc = dict(o_del=5, e_del=2, o_ins=7, e_ins=1, zdrop=50, end_bonus=3, a=2, b=3)
    e = bsw.Engine(_gparams(sc), small_batch=0, mid_batch=0)
    pairs, ref, qer = bswgen.random_pairs(2000, seed=31, tlen=(0, 300), qlen=(0, 160))
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(sc), want, ref, qer, 60, nthreads=8)
    e.get_scores(got, ref, qer, 60)
    _assert_same(want, got, "alt scoring")


@pytest.fixture(scope="module")
def c2_full():
    pairs, ref, qer = bsw.synth_batch(1_000_000)
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=16)
    return pairs, ref, qer, want


def test_c2_full_workload_device_api(eng, c2_full):
    pairs, ref, qer, want = c2_full
    dp = hiprt.DeviceBuffer.from_array(pairs)
    dr = hiprt.DeviceBuffer.from_array(ref)
    dq = hiprt.DeviceBuffer.from_array(qer)
    eng.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), 100)
    got = dp.download(np.empty_like(pairs))
    _assert_same(want, got, "C2 1M device API")
    # idempotence: a second pass over the same resident batch changes nothing
    eng.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), 100)
    again = dp.download(np.empty_like(pairs))
    assert np.array_equal(got, again)


def test_c2_full_workload_host_api_permuted(eng, c2_full):
    pairs, ref, qer, want = c2_full
    perm = np.random.default_rng(5).permutation(len(pairs))
    got = pairs[perm].copy()
    eng.get_scores(got, ref, qer, 100)
    _assert_same(want[perm], got, "C2 1M permuted host API")
    # inputs untouched
    for f in ("idr", "idq", "id", "len1", "len2", "h0", "seqid", "regid"):
        assert np.array_equal(got[f], pairs[perm][f])


def test_cell_bits_8_matches_16(eng, c2_full):
    """getScores8 path: every C2 pair is in the 8-bit score regime (h0 + 150 <= 255) and takes
    the packed kernel (n_u8); results equal the int16 path's / the oracle's."""
    pairs, ref, qer, want = c2_full
    got = pairs[:200_000].copy()
    eng.get_scores(got, ref, qer, 100, cell_bits=8)
    _assert_same(want[:200_000], got, "cell_bits=8")
    st = eng.last_stats()
    assert st.n_u8 == 200_000 and st.n_i16 == 0


def test_cell_bits_8_overflow_fallback(eng):
    """C3-style routing: pairs whose score could exceed 255 fall back to the int16 kernels."""
    pairs, ref, qer = bswgen.random_pairs(5000, seed=33, qlen=(0, 170), tlen=(0, 330), h0=(0, 200))
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    eng.get_scores(got, ref, qer, 100, cell_bits=8)
    _assert_same(want, got, "cell_bits=8 mixed")
    st = eng.last_stats()
    q, t, h0 = pairs["len2"], pairs["len1"], pairs["h0"]
    narrow = (q < 160) & (h0 + np.minimum(q, t) <= 255)      # packed-column kernel: qlen < QMAX
    assert st.n_u8 == int(narrow.sum())
    assert st.n_i16 + st.n_wide == len(pairs) - int(narrow.sum())


def test_concurrent_callers(eng):
    batches = [bswgen.random_pairs(1500, seed=900 + k) for k in range(4)]
    wants, gots, errs = [], [], []
    for pairs, ref, qer in batches:
        w_ = pairs.copy()
        oracle.get_scores(_oparams(), w_, ref, qer, 100, nthreads=4)
        wants.append(w_)
        gots.append(pairs.copy())

    def run(k):
        try:
            for _ in range(3):
                eng.get_scores(gots[k], batches[k][1], batches[k][2], 100)
        except Exception as ex:  # noqa: BLE001
            errs.append(ex)

    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs
    for k in range(4):
        _assert_same(wants[k], gots[k], f"thread {k}")


@pytest.mark.parametrize("chunk", [1, 8192, 1 << 20])
def test_host_pipeline_chunks(chunk):
    """Host-buffer pipeline (bsw_get_scores): the batch is staged / copied / computed chunk by
    chunk over two slots (BSW_OPT_HOST_CHUNK); contiguous batches stage byte extents in bulk,
    permuted ones are gathered pair by pair with rewritten offsets.  Chunks are whole 4096-pair
    blocks: chunk 1 and 8192 give 3 and 3 chunks, 1 << 20 one.  Outputs equal the oracle and
    only the six output fields of the caller's records change."""
    e = bsw.Engine(host_chunk=chunk, small_batch=0, mid_batch=0)
    pairs, ref, qer = bswgen.random_pairs(20000 if chunk > 1 else 9000, seed=chunk % 1000, qlen=(0, 190), tlen=(0, 330))
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    for order in (np.arange(len(pairs)), np.random.default_rng(chunk).permutation(len(pairs))):
        got = pairs[order].copy()
        e.get_scores(got, ref, qer, 100)
        _assert_same(want[order], got, f"chunk {chunk}")
        for f in ("idr", "idq", "id", "len1", "len2", "h0", "seqid", "regid"):
            assert np.array_equal(got[f], pairs[order][f])
    e.close()


@pytest.mark.parametrize("chunk", [4096, 65536, 262144])
def test_host_pipeline_chunks_equal_oracle(chunk, c2_full):
    """The host pipeline (bsw_host.cpp host_shard: 2-bit staging, H2D, device unpack / plan / sort,
    DP, 24-B outputs back) over contiguous C2 batches with extra N bases, empty sequences and the
    8-bit regime's edge h0 values, in 1 to ~75 chunks (chunks of <= 32K pairs take the row-group
    kernel); outputs equal the oracle and only the six output fields change."""
    pairs, ref, qer, _ = c2_full
    n = 300_000
    p = pairs[:n].copy()
    r, q = ref.copy(), qer.copy()
    q[13::997] = 4                                   # more N than C2 has (codes are 0..4 by the ABI)
    r[5::1201] = 4
    p["len2"][::5001] = 0                            # empty queries / targets
    p["len1"][3::7001] = 0
    qs = p["len2"] > 0
    p["h0"][qs & (np.arange(n) % 13 == 0)] = 255 - np.minimum(p["len2"], p["len1"])[qs & (np.arange(n) % 13 == 0)]
    want = p.copy()
    oracle.get_scores(_oparams(), want, r, q, 100, nthreads=16)
    e = bsw.Engine(host_chunk=chunk)
    got = p.copy()
    e.get_scores(got, r, q, 100)
    _assert_same(want, got, f"fast path chunk {chunk}")
    for f in ("idr", "idq", "id", "len1", "len2", "h0", "seqid", "regid"):
        assert np.array_equal(got[f], p[f])
    st = e.last_stats()
    assert st.n_packed + st.n_group == n and st.n_launches >= 1
    e.close()


@pytest.mark.parametrize("bad_at", [10, 150_000, 199_999])
def test_host_pipeline_invalid_pair_writes_nothing(bad_at):
    """The pipeline validates the first chunk's blocks, starts it, and validates the rest before
    any chunk's outputs are written back: an invalid pair anywhere (first chunk, middle, last
    pair) returns BSW_E_RANGE with every caller record unchanged.  Then the same engine scores the
    repaired batch (remainder chunk merged into the last one) equal to the oracle."""
    e = bsw.Engine(host_chunk=65536, small_batch=0, mid_batch=0)
    pairs, ref, qer = bsw.synth_batch(200_000, pair_base=77)
    bad = pairs.copy()
    bad[bad_at]["len1"] = -1
    before = bad.copy()
    with pytest.raises(bsw.BswError, match="-34"):
        e.get_scores(bad, ref, qer, 100)
    assert np.array_equal(bad, before)
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=16)
    got = pairs.copy()
    e.get_scores(got, ref, qer, 100)
    _assert_same(want, got, f"after the rejected call (bad_at={bad_at})")
    e.close()


@pytest.mark.parametrize("pack,p_n", [(2, 0.0), (2, 0.02), (2, 0.1), (4, 0.02)])
def test_host_pipeline_packing(pack, p_n):
    """Staging of contiguous sequence buffers (BSW_OPT_HOST_PACK): 2-bit codes + exception words
    for N bytes, 20-B input records and 24-B outputs back (default), or nibbles + whole records.
    p_n = 0.1 puts more than 1/32 of the bytes outside 0..3, so those chunks fall back to nibbles.
    Odd extents (lengths 0..331) exercise the unpack tails; outputs equal the oracle either way and
    the caller's input fields are untouched."""
    e = bsw.Engine(host_chunk=8192, host_pack=pack, small_batch=0, mid_batch=0)
    pairs, ref, qer = bswgen.random_pairs(20000, seed=int(p_n * 1000) + pack, qlen=(0, 190), tlen=(0, 331), p_n=p_n)
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    got = pairs.copy()
    e.get_scores(got, ref, qer, 100)
    _assert_same(want, got, f"pack {pack} p_n {p_n}")
    for f in ("idr", "idq", "id", "len1", "len2", "h0", "seqid", "regid"):
        assert np.array_equal(got[f], pairs[f])
    e.close()


@pytest.mark.parametrize("group", [1, 0])
@pytest.mark.parametrize("n", [1, 63, 1000, 16384, 16385, 32768, 32769])
def test_small_batch_route(n, group, c2_full):
    """Default routing (BSW_OPT_SMALL_BATCH = BSW_OPT_MID_BATCH = 32768): calls of at most 32768
    pairs run on the row-group kernel (16 lanes per pair, no plan / sort; BSW_OPT_GROUP_KERNEL 1) or,
    with it off, every int16-safe pair on the wave-per-alignment kernel; larger calls on the lane /
    packed-column classes.  Both entry points (host buffers, resident) and both cell widths give
    the oracle's outputs."""
    pairs, ref, qer, want = c2_full
    e = bsw.Engine(group_kernel=group)
    small = n <= 32768
    rg = group and n <= 32768
    for cell_bits in (16, 8):
        got = pairs[:n].copy()
        e.get_scores(got, ref, qer, 100, cell_bits)
        _assert_same(want[:n], got, f"n {n} cell_bits {cell_bits}")
        st = e.last_stats()
        assert st.n_group == (n if rg else 0)
        assert st.n_wave == (n if small and not group else 0)
        assert st.n_i16 + st.n_u8 + st.n_wide == n
    dp, dr, dq = (hiprt.DeviceBuffer.from_array(a) for a in (pairs[:n].copy(), ref, qer))
    e.get_scores_device(dp.ptr, dr.ptr, dq.ptr, n, 100, 16)
    _assert_same(want[:n], dp.download(np.empty_like(pairs[:n])), f"device n {n}")
    assert e.last_stats().n_group == (n if rg else 0)
    e.close()


@pytest.mark.parametrize("w", [0, 7, 100, 200])
def test_group_kernel_quad_random(w):
    """The quad form of the row-group kernel (4 lanes per pair; BSW_OPT_SMALL_BATCH 0 sends every
    batch of up to BSW_OPT_MID_BATCH pairs there): random shapes with targets up to its 512 bytes
    and a few past them (the batch then takes the planned path), both entry points."""
    e = bsw.Engine(small_batch=0)
    pairs, ref, qer = bswgen.random_pairs(6000, seed=1900 + w, tlen=(0, 512), qlen=(0, 160), h0=(0, 200))
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
    got = pairs.copy()
    e.get_scores(got, ref, qer, w)
    _assert_same(want, got, f"quad host w={w}")
    assert e.last_stats().n_group == len(pairs)
    dp, dr, dq = (hiprt.DeviceBuffer.from_array(a) for a in (pairs.copy(), ref, qer))
    e.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), w, 16)
    _assert_same(want, dp.download(np.empty_like(pairs)), f"quad device w={w}")
    assert e.last_stats().n_group == len(pairs)
    long_t, r2, q2 = bswgen.random_pairs(3000, seed=2900 + w, tlen=(400, 700), qlen=(0, 160), h0=(0, 200))
    want2 = long_t.copy()
    oracle.get_scores(_oparams(), want2, r2, q2, w, nthreads=8)
    got2 = long_t.copy()
    e.get_scores(got2, r2, q2, w)
    _assert_same(want2, got2, f"quad fallback host w={w}")
    dp, dr, dq = (hiprt.DeviceBuffer.from_array(a) for a in (long_t.copy(), r2, q2))
    e.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(long_t), w, 16)
    _assert_same(want2, dp.download(np.empty_like(long_t)), f"quad fallback device w={w}")
    e.close()


@pytest.mark.parametrize("w", [0, 1, 7, 100, 200])
def test_group_kernel_random(w):
    """The row-group kernel over random shapes (queries 0..160, targets 0..400, h0 0..200),
    both entry points: host buffers (host-checked contract) and device buffers (kernel-checked,
    flag read back)."""
    e = bsw.Engine()
    pairs, ref, qer = bswgen.random_pairs(3000, seed=900 + w, tlen=(0, 400), qlen=(0, 160), h0=(0, 200))
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
    got = pairs.copy()
    e.get_scores(got, ref, qer, w)
    _assert_same(want, got, f"group kernel host w={w}")
    assert e.last_stats().n_group == len(pairs)
    dp, dr, dq = (hiprt.DeviceBuffer.from_array(a) for a in (pairs.copy(), ref, qer))
    e.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), w, 16)
    _assert_same(want, dp.download(np.empty_like(pairs)), f"group kernel device w={w}")
    assert e.last_stats().n_group == len(pairs)
    e.close()


@pytest.mark.parametrize("quad", [False, True])
def test_group_kernel_golden(golden, quad, monkeypatch):
    """Every golden batch on the default engine (small batches: the row-group kernel where the
    scoring qualifies, the planned path otherwise) and on the device entry point; quad: every
    batch on the 4-lanes-per-pair form (BSW_OPT_SMALL_BATCH 0).  The 16-lane form here
    (BSW_OPT_GQ32_MAX 0: batches of <= 2048 pairs would take the 32-lane form, tested on its own)."""
    engines, ran = {}, 0
    for name, pairs, ref, qer, w, sc in golden:
        key = tuple(sorted(sc.items()))
        if key not in engines:
            engines[key] = bsw.Engine(_gparams(sc), gq32_max=0, **({"small_batch": 0} if quad else {}))
        got = pairs.copy()
        for f in bsw.OUT_FIELDS:
            got[f] = -9
        engines[key].get_scores(got, ref, qer, w)
        _assert_same(pairs, got, f"golden {name} default route")
        ran += engines[key].last_stats().n_group
        dev = pairs.copy()
        for f in bsw.OUT_FIELDS:
            dev[f] = -9
        dp, dr, dq = (hiprt.DeviceBuffer.from_array(a) for a in (dev, ref, qer))
        engines[key].get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), w, 16)
        _assert_same(pairs, dp.download(np.empty_like(pairs)), f"golden {name} device route")
    assert ran > 0
    for e in engines.values():
        e.close()


@pytest.mark.parametrize("w", [5, 100])
def test_group_kernel_score_255_boundary(w, monkeypatch):
    """The row-group kernel's 8-bit row-max key (bsw_gq.hip, K8: H << 8 | j in 16 bits) holds only
    when every live pair of the wave has h0 + min(qlen, tlen) <= 255.  Identical query / target
    pairs with h0 = 255 - qlen drive H to exactly 255 on the diagonal; waves of four pairs (16
    lanes each) mix them with pairs at h0 + qlen = 256 (the wave then runs the 16-bit key) and
    with near-identical ones, in every position of the wave.  Host and device entry points, both
    routed to the 16-lane form (BSW_OPT_GQ32_MAX 0), equal the oracle."""
    rng = np.random.default_rng(255 + w)
    items = []
    for k in range(64):
        qlen = int(rng.choice([40, 100, 149, 150, 159, 160]))
        q = rng.integers(0, 4, qlen).astype(np.uint8)
        t = np.concatenate([q, rng.integers(0, 4, int(rng.integers(0, 140))).astype(np.uint8)])
        over = (k // 4) % 3          # wave k // 4: all at 255 / one at 256 / all at 256
        h0 = 255 - qlen + (1 if over == 2 or (over == 1 and k % 4 == (k // 12) % 4) else 0)
        if k % 5 == 4:               # a mismatch somewhere: H stays below the bound
            j = int(rng.integers(0, qlen))
            q = q.copy()
            q[j] = (q[j] + 1) & 3
        items.append((t, q, h0))
    pairs, ref, qer = bswgen.assemble(items)
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
    assert (want["score"] == 255).sum() >= 8 and (want["score"] == 256).sum() >= 8
    e = bsw.Engine(gq32_max=0)
    for cell_bits in (16, 8):
        got = pairs.copy()
        e.get_scores(got, ref, qer, w, cell_bits)
        _assert_same(want, got, f"gq 255/256 host w={w} cell_bits={cell_bits}")
        assert e.last_stats().n_group == len(pairs)
    dp, dr, dq = (hiprt.DeviceBuffer.from_array(a) for a in (pairs.copy(), ref, qer))
    e.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), w, 16)
    _assert_same(want, dp.download(np.empty_like(pairs)), f"gq 255/256 device w={w}")
    assert e.last_stats().n_group == len(pairs)
    e.close()


@pytest.mark.parametrize("n", [0, 1, 700, 40_000])
def test_packed_device_equal_oracle(n):
    """bsw_get_scores_packed_device: a batch in the 2-bit wire form (bsw_pack_batch: 20-B records,
    2-bit codes, exception words for N and other non-ACGT bytes) uploaded as one buffer, unpacked
    on the device and scored; the 24 output bytes per pair equal the oracle.  Small batches take
    the row-group kernel, 40K pairs the planned path; mixed shapes include long queries and
    int16-unsafe h0 (several kernel classes)."""
    pairs, ref, qer = bswgen.random_pairs(max(n, 1), seed=600 + n, qlen=(0, 300), tlen=(0, 400), h0=(0, 300))
    pairs = pairs[:n]
    qer[7::61] = 4
    ref[3::89] = 4
    if n > 100:
        pairs["h0"][::37] = 32000
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    buf, d = bsw.pack_batch(pairs, ref, qer)
    db = hiprt.DeviceBuffer.from_array(buf)
    out = np.full((max(n, 1), 6), -7, dtype=np.int32)
    dout = hiprt.DeviceBuffer.from_array(out)
    e = bsw.Engine()
    for cell_bits in (16, 8):
        e.get_scores_packed_device(db.ptr, d, 100, cell_bits, dout.ptr)
        got = dout.download(np.empty_like(out))[:n]
        for k, f in enumerate(bsw.OUT_FIELDS):
            bad = int((got[:, k] != want[f]).sum())
            assert bad == 0, f"packed n={n} cell_bits={cell_bits}: {f} differs in {bad} pairs"
    e.close()


def test_packed_device_dense_exceptions():
    """The staging kernel's exception walk past one 64-word round: runs of thousands of N in the
    reference and the queries (every word of a wave's 4096 positions is an exception), N at a
    segment's first and last positions, and exceptions in only one of the two buffers."""
    pairs, ref, qer = bswgen.random_pairs(20_000, seed=777, qlen=(0, 160), tlen=(0, 300), h0=(0, 120))
    for case in range(3):
        r, q = ref.copy(), qer.copy()
        if case != 2:
            r[5000:17000] = 4                                 # 12K consecutive exception words
            r[0] = 4
            r[-1] = 4
        if case != 1:
            q[2000:9000] = 4
            q[-1] = 4
        want = pairs.copy()
        oracle.get_scores(_oparams(), want, r, q, 100, nthreads=8)
        buf, d = bsw.pack_batch(pairs, r, q)
        db = hiprt.DeviceBuffer.from_array(buf)
        out = np.full((len(pairs), 6), -7, dtype=np.int32)
        dout = hiprt.DeviceBuffer.from_array(out)
        e = bsw.Engine()
        e.get_scores_packed_device(db.ptr, d, 100, 16, dout.ptr)
        got = dout.download(np.empty_like(out))
        for k, f in enumerate(bsw.OUT_FIELDS):
            bad = int((got[:, k] != want[f]).sum())
            assert bad == 0, f"dense exceptions case {case}: {f} differs in {bad} pairs"
        e.close()


def test_group_kernel_fallback_device():
    """Device entry point, small batch with a few pairs outside the row-group contract (query past
    160, int16-unsafe h0): the kernel flags them and the whole batch reruns on the planned path."""
    pairs, ref, qer = bswgen.random_pairs(2000, seed=4242, tlen=(0, 400), qlen=(0, 160), h0=(0, 200))
    pairs["h0"][7] = 32000
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    e = bsw.Engine()
    dp, dr, dq = (hiprt.DeviceBuffer.from_array(a) for a in (pairs.copy(), ref, qer))
    e.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), 100, 16)
    _assert_same(want, dp.download(np.empty_like(pairs)), "group kernel fallback")
    st = e.last_stats()
    assert st.n_group == 0 and st.n_i16 + st.n_u8 + st.n_wide == len(pairs)
    e.close()


def test_small_batch_mixed():
    """A small batch holding int16-unsafe pairs (h0 large) and queries past 160 columns: the
    unsafe ones stay on the int32 wide kernel, most of the rest go to the wave kernel (empty
    pairs keep their lane class)."""
    pairs, ref, qer = bswgen.random_pairs(3000, seed=91, qlen=(0, 400), tlen=(0, 500), h0=(0, 32700))
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    e = bsw.Engine()
    got = pairs.copy()
    e.get_scores(got, ref, qer, 100)
    _assert_same(want, got, "mixed small batch")
    st = e.last_stats()
    assert st.n_wide > 0 and st.n_wave > 0 and st.n_i16 + st.n_u8 + st.n_wide == len(pairs)
    e.close()


def test_multi_gpu_context_shards(c2_full):
    pairs, ref, qer, want = c2_full
    n = hiprt.device_count()
    e = bsw.Engine(n_gpus=n, small_batch=0, mid_batch=0)
    got = pairs[:100_000].copy()
    e.get_scores(got, ref, qer, 100)
    _assert_same(want[:100_000], got, f"n_gpus={n}")


@pytest.mark.parametrize("nlog", [2, 4])
def test_multi_device_policy_rehearsal(c2_full, nlog):
    """A context of nlog logical devices on the box's one GPU (bsw_create_on with a repeated
    device, the rehearsal of an nlog-GPU node): calls below BSW_OPT_SPLIT_MIN run whole on one
    device (n_devices == 1), larger calls split over all of them, split_min = 0 splits every
    call; 8 concurrent callers of 1K / 10K pairs; mate-rescue and global calls through the same
    policy -- all equal the oracle."""
    pairs, ref, qer, want = c2_full
    e = bsw.Engine(devices=[0] * nlog)
    for m, nd in ((1000, 1), (10_000, 1), (200_000, nlog)):
        got = pairs[:m].copy()
        e.get_scores(got, ref, qer, 100)
        _assert_same(want[:m], got, f"{nlog} logical devices, {m} pairs")
        assert e.last_stats().n_devices == nd
    e.set_option("split_min", 0)
    got = pairs[:3000].copy()
    e.get_scores(got, ref, qer, 100)
    _assert_same(want[:3000], got, f"{nlog} logical devices, forced split")
    assert e.last_stats().n_devices == nlog
    e.set_option("split_min", 131072)
    errs = []

    def caller(k, m):
        try:
            for r in range(4):
                a = ((k * 4 + r) * m) % (len(pairs) - m)
                got = pairs[a:a + m].copy()
                e.get_scores(got, ref, qer, 100, 8 if r & 1 else 16)
                _assert_same(want[a:a + m], got, f"caller {k} round {r}")
        except Exception as x:  # noqa: BLE001
            errs.append(x)
    for m in (1000, 10_000):
        th = [threading.Thread(target=caller, args=(k, m)) for k in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    assert not errs, errs[0]
    mref = bsw.synth_reference(400_000, seed=9)
    mp, mq = bsw.synth_mates(mref, 3000)
    mwant = oracle.ksw_align2_batch(mp, mref, mq, bwa_fill_scmat(), nthreads=8)
    ref_one = bsw.Engine()
    for w_split in (131072, 0):
        e.set_option("split_min", w_split)
        got = bsw.ksw_align2(e, mp, mref, mq)
        assert np.array_equal(got, bsw.ksw_align2(ref_one, mp, mref, mq))
        for f in ("score", "te", "qe"):
            assert np.array_equal(got[f], mwant[f]), f
    e.close()
    ref_one.close()


@pytest.fixture(scope="module")
def eng_lane():
    """Engine with the packed-column kernel disabled (BSW_OPT_KERNEL8 = 0): every pair runs on
    the int16 lane kernel (bsw_kernels.hip) or the wide kernel."""
    e = bsw.Engine(kernel8=0, small_batch=0, mid_batch=0)
    yield e
    e.close()


@pytest.mark.parametrize("w", [0, 1, 7, 40, 100, 200])
def test_pc_kernel_random(eng, w):
    """8-bit-regime pairs (h0 + min(qlen, tlen) <= 255, qlen < 160) run on bsw_pc.hip."""
    pairs, ref, qer = bswgen.random_pairs(6000, seed=170 + w, qlen=(0, 159), tlen=(0, 330), h0=(0, 95))
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
    eng.get_scores(got, ref, qer, w)
    _assert_same(want, got, f"pc w={w}")
    assert eng.last_stats().n_packed == len(pairs)


@pytest.mark.parametrize("cell_bits", [16, 8])
def test_pc_kernel_bucket_edges(eng, cell_bits):
    """qlen at every bucket edge (31/32/33 ... 159/160/161: 160 goes to the lane kernel,
    161 to the wide kernel), h0 at the 8-bit bound, tiny and long targets."""
    rng = np.random.default_rng(11)
    shapes = []
    for q in (0, 1, 2, 3, 4, 5, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 159, 160, 161):
        for t in (0, 1, 3, q, q + 1, 2 * q + 7, 300):
            h0 = int(min(rng.integers(0, 120), max(0, 255 - min(q, t))))
            shapes.append((t, q, h0))
            shapes.append((t, q, max(0, 255 - min(q, t))))         # exactly at the bound
            shapes.append((t, q, 256 - min(q, t)))                 # one above: lane kernel
    pairs, ref, qer = bswgen.pairs_from_shapes(shapes, seed=12)
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    eng.get_scores(got, ref, qer, 100, cell_bits=cell_bits)
    _assert_same(want, got, f"pc bucket edges cb={cell_bits}")
    assert eng.last_stats().n_packed > 0


@pytest.mark.parametrize("q", [4, 5, 6, 7, 8, 64, 97, 148, 149, 150, 151, 158])
@pytest.mark.parametrize("w", [3, 100])
def test_pc_kernel_qlen_tail(eng, q, w):
    """Waves of one qlen whose rows all end at qlen run the qlen-tail group body (FAST body,
    key limited to slots <= qlen, h1 from slot qlen): every residue qlen & 3, related reads
    (the synthetic C2 generator) so the band reaches qlen, a narrow and the C2 band."""
    cfg = bsw.synth_cfg(qlen=q, tlen=2 * q + 3, h0_lo=0, h0_hi=min(95, 255 - q))
    pairs, ref, qer = bsw.synth_batch(8192, pair_base=1000 * q + w, cfg=cfg)
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
    eng.get_scores(got, ref, qer, w)
    _assert_same(want, got, f"qlen tail q={q} w={w}")
    assert eng.last_stats().n_packed == len(pairs)


def test_lane_kernel_random(eng_lane):
    pairs, ref, qer = bswgen.random_pairs(6000, seed=77, qlen=(0, 160), tlen=(0, 330), h0=(0, 95))
    want, got = pairs.copy(), pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    eng_lane.get_scores(got, ref, qer, 100)
    _assert_same(want, got, "lane kernel random")
    assert eng_lane.last_stats().n_packed == 0


def test_lane_kernel_c2(eng_lane, c2_full):
    pairs, ref, qer, want = c2_full
    got = pairs[:300_000].copy()
    eng_lane.get_scores(got, ref, qer, 100)
    _assert_same(want[:300_000], got, "lane kernel C2")
    assert eng_lane.last_stats().n_packed == 0


def test_argument_errors(eng):
    pairs, ref, qer = bswgen.random_pairs(10, seed=1)
    lib = bsw.hip_lib()
    import ctypes
    P = ctypes.c_void_p
    assert lib.bsw_get_scores(eng._ctx, P(pairs.ctypes.data), P(ref.ctypes.data), P(qer.ctypes.data),
                              -1, 100, 16) == -22
    assert lib.bsw_get_scores(eng._ctx, P(pairs.ctypes.data), P(ref.ctypes.data), P(qer.ctypes.data),
                              10, -1, 16) == -22
    assert lib.bsw_get_scores(eng._ctx, P(pairs.ctypes.data), P(ref.ctypes.data), P(qer.ctypes.data),
                              10, 100, 12) == -22
    bad = pairs.copy()
    bad["len1"][3] = 40000
    assert lib.bsw_get_scores(eng._ctx, P(bad.ctypes.data), P(ref.ctypes.data), P(qer.ctypes.data),
                              10, 100, 16) == -34
    # empty batch is a no-op
    eng.get_scores(pairs[:0].copy(), ref, qer, 100)


def test_kernel_range_guard_reports_error():
    """BSW_OPT_TEST_MISROUTE sends every pair to the QMAX=32 lane kernel: pairs with longer
    queries trip the kernel's range guard, and both call forms must return BSW_E_RANGE (the
    guard word is read back after the DP launches) instead of BSW_OK with unwritten outputs."""
    pairs, ref, qer = bswgen.c2_like(500, seed=41)
    e = bsw.Engine(test_misroute=1, small_batch=0, mid_batch=0)
    got = pairs.copy()
    with pytest.raises(bsw.BswError, match="-34"):
        e.get_scores(got, ref, qer, 100)
    dp = hiprt.DeviceBuffer.from_array(pairs)
    dr = hiprt.DeviceBuffer.from_array(ref)
    dq = hiprt.DeviceBuffer.from_array(qer)
    with pytest.raises(bsw.BswError, match="-34"):
        e.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), 100)
    # short queries fit the QMAX=32 class: the same misrouted engine returns the oracle's results
    sp, sr, sq = bswgen.random_pairs(800, seed=42, qlen=(0, 32), tlen=(0, 90))
    want, got = sp.copy(), sp.copy()
    oracle.get_scores(_oparams(), want, sr, sq, 100)
    e.get_scores(got, sr, sq, 100)
    _assert_same(want, got, "misrouted short queries")
    # a multi-chunk host call (launcher-thread pipeline): the guard trips inside the pipeline,
    # the call returns BSW_E_RANGE without hanging, and the engine keeps working afterwards
    big, bref, bqer = bswgen.c2_like(40_000, seed=43)
    e.set_option("host_chunk", 4096)
    with pytest.raises(bsw.BswError, match="-34"):
        e.get_scores(big.copy(), bref, bqer, 100)
    e.set_option("test_misroute", 0)
    got = pairs.copy()
    e.get_scores(got, ref, qer, 100)
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100)
    _assert_same(want, got, "after a tripped guard")
    gb, wb = big.copy(), big.copy()
    e.get_scores(gb, bref, bqer, 100)
    oracle.get_scores(_oparams(), wb, bref, bqer, 100)
    _assert_same(wb, gb, "chunked call after a tripped guard")
    e.close()


def test_options_api(eng):
    lib = bsw.hip_lib()
    assert lib.bsw_set_option(eng._ctx, 999, 1) == -22
    assert lib.bsw_set_option(eng._ctx, bsw.OPT_FORK, 2) == -22
    assert lib.bsw_set_option(eng._ctx, bsw.OPT_EXT_CHUNK, -1) == -22
    assert lib.bsw_set_option(None, bsw.OPT_FORK, 1) == -22
    assert lib.bsw_set_option(eng._ctx, bsw.OPT_SORTKEY, 1) == 0
    assert lib.bsw_set_option(eng._ctx, bsw.OPT_KERNEL8, 3) == -22          # 0, 1, 2 only
    assert lib.bsw_set_option(eng._ctx, 15, 0) == -22                       # removed in ABI 8
    assert lib.bsw_set_option(eng._ctx, 17, 0) == -22                       # removed in ABI 8
    assert lib.bsw_set_option(eng._ctx, 16, 100001) == -22                  # BSW_OPT_COALESCE_LINGER
    assert lib.bsw_set_option(eng._ctx, 16, 30) == 0
    assert lib.bsw_set_option(eng._ctx, bsw.OPT_GQ32_MAX, -1) == -22
    assert lib.bsw_set_option(eng._ctx, bsw.OPT_GQ32_MAX, 2048) == 0


@pytest.mark.parametrize("gaps", [(100, 16400, 6, 1), (6, 1, 30000, 2700), (16000, 16000, 16000, 16000)])
def test_extreme_gap_penalties(gaps):
    """Legal but extreme gap penalties (o + e up to 32767) on the default (small-batch) routing
    and with every eligible pair forced to the wave kernel: the wave kernel's int16 E/F lanes
    must not see them (wv_class bound), results equal the oracle."""
    o_del, e_del, o_ins, e_ins = gaps
    sc = dict(a=1, b=4, o_del=o_del, e_del=e_del, o_ins=o_ins, e_ins=e_ins, zdrop=100, end_bonus=5)
    pairs, ref, qer = bswgen.random_pairs(1500, seed=sum(gaps), tlen=(0, 320), qlen=(0, 200))
    want = pairs.copy()
    oracle.get_scores(_oparams(sc), want, ref, qer, 100, nthreads=8)
    for opts in ({}, {"long": 2}):
        e = bsw.Engine(_gparams(sc), **opts)
        got = pairs.copy()
        e.get_scores(got, ref, qer, 100)
        _assert_same(want, got, f"gaps {gaps} {opts}")
        assert e.last_stats().n_wave == 0
        e.close()


def test_host_pipeline_2bit_pieces_over_8mb():
    """One staged chunk spanning ~19 MB of reference and ~11 MB of query bytes, so stage_2bit
    splits both buffers into several parallel pieces (cuts at multiples of 64 codes, 4 MB
    apart): N bases sit on both sides of every 64-code boundary (positions 0 and 63 mod 64 of
    the 64-aligned sequences), so each piece's AVX2/SSE tail and its exception words' offsets
    (pos0) are exercised.  2-bit staging and nibble staging both equal the oracle."""
    rng = np.random.default_rng(64)
    n, TS, QS = 60_000, 320, 192
    ref = rng.integers(0, 4, n * TS, dtype=np.uint8)
    qer = np.zeros(n * QS, dtype=np.uint8)
    pairs = np.zeros(n, dtype=oracle.SEQPAIR_DTYPE)
    idx = np.arange(n)
    pairs["idr"], pairs["idq"] = idx * TS, idx * QS
    pairs["len1"], pairs["len2"], pairs["id"] = 300, 150, idx
    pairs["h0"] = rng.integers(19, 100, n)
    q = ref.reshape(n, TS)[:, :150].copy()
    mut = rng.random(q.shape) < 0.02
    q[mut] = (q[mut] + rng.integers(1, 4, int(mut.sum()))) % 4
    qer.reshape(n, QS)[:, :150] = q
    pos = np.arange(len(ref))
    ref[(pos % 64 == 0) | (pos % 64 == 63)] = 4
    qpos = np.arange(len(qer))
    qer[(qpos % 128 == 0) | (qpos % 128 == 127)] = 4
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, 100, nthreads=8)
    for pack in (2, 4):
        e = bsw.Engine(host_chunk=1 << 17, host_pack=pack, small_batch=0, mid_batch=0)
        got = pairs.copy()
        e.get_scores(got, ref, qer, 100)
        _assert_same(want, got, f"pieces > 8 MB, host_pack {pack}")
        e.close()


def test_coalesced_small_calls(c2_full):
    """Cross-call coalescing (BSW_OPT_COALESCE): 8 kt_for-style threads issue small calls of
    varying sizes, w and cell_bits -- some with scattered (non-contiguous) buffers, one with a pair
    past BSW_MAX_LEN -- concurrently on one context; every call returns its own outputs (== the
    oracle), the bad call alone gets BSW_E_RANGE, and coalescing off gives the same; a long leader
    linger (BSW_OPT_COALESCE_LINGER 3000 us: other leaders take the lingering caller's request
    meanwhile) and none give the same too."""
    pairs, ref, qer, want = c2_full
    want200 = None
    for co, linger in ((32768, 30), (32768, 3000), (32768, 0), (0, 30)):
        e = bsw.Engine(coalesce=co, coalesce_linger=linger)
        errs, bad_seen = [], []
        rng = np.random.default_rng(7)
        plan = [[(int(rng.integers(0, len(pairs) - 60000)), int(rng.choice([1, 57, 1000, 3000, 10000, 20000])),
                  int(rng.choice([100, 200])), int(rng.choice([16, 8]))) for _ in range(12)] for _ in range(8)]

        def caller(k):
            try:
                for j, (a, m, w, cb) in enumerate(plan[k]):
                    got = pairs[a:a + m].copy()
                    if k == 3 and j == 5:                       # one bad call among them
                        got[m // 2]["len1"] = 40000
                        with pytest.raises(bsw.BswError):
                            e.get_scores(got, ref, qer, w, cb)
                        bad_seen.append(1)
                        continue
                    if k == 5 and j % 3 == 0:                   # scattered: every 3rd pair of a range
                        got = pairs[a:a + 3 * m:3].copy()       # (extents 3x the bytes: not bulk)
                        wv = want[a:a + 3 * m:3]
                    else:
                        wv = want[a:a + m]
                    e.get_scores(got, ref, qer, w, cb)
                    if w == 100:
                        _assert_same(wv, got, f"caller {k} call {j}")
                    else:
                        ref_out = got.copy()
                        oracle.get_scores(_oparams(), ref_out, ref, qer, w, nthreads=2)
                        _assert_same(ref_out, got, f"caller {k} call {j} w {w}")
            except Exception as x:  # noqa: BLE001
                errs.append(x)
        th = [threading.Thread(target=caller, args=(k,)) for k in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs[0]
        assert bad_seen == [1]
        e.close()


@pytest.mark.parametrize("w", [0, 1, 7, 100, 200])
def test_group_kernel_32lane(w):
    """The row-group kernel's 32-lane latency form (bsw_gq.hip GS = 32: two DPP rows per pair, scans
    closed by row_bcast:15, the column shift by wave_shr:1, reductions by v_permlane16_swap), routed
    by BSW_OPT_GQ32_MAX: random shapes (queries 0..160 -> 2 / 4 / 6 columns per lane,
    targets 0..400, h0 0..200), the 255/256 key boundary, host and device entry points == oracle."""
    e = bsw.Engine(gq32_max=1_000_000)
    for qhi in (60, 120, 160):
        pairs, ref, qer = bswgen.random_pairs(3000, seed=7100 + w + qhi, tlen=(0, 400), qlen=(0, qhi), h0=(0, 200))
        want = pairs.copy()
        oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
        got = pairs.copy()
        e.get_scores(got, ref, qer, w)
        _assert_same(want, got, f"gq32 host w={w} qlen<={qhi}")
        assert e.last_stats().n_group == len(pairs)
        dp, dr, dq = (hiprt.DeviceBuffer.from_array(a) for a in (pairs.copy(), ref, qer))
        e.get_scores_device(dp.ptr, dr.ptr, dq.ptr, len(pairs), w, 16)
        _assert_same(want, dp.download(np.empty_like(pairs)), f"gq32 device w={w} qlen<={qhi}")
        assert e.last_stats().n_group == len(pairs)
    rng = np.random.default_rng(3255 + w)
    items = []
    for k in range(64):
        qlen = int(rng.choice([40, 100, 150, 159, 160]))
        q = rng.integers(0, 4, qlen).astype(np.uint8)
        t = np.concatenate([q, rng.integers(0, 4, int(rng.integers(0, 140))).astype(np.uint8)])
        h0 = 255 - qlen + ((k // 2) % 2)          # waves of two pairs: at 255 / at 256
        items.append((t, q, h0))
    pairs, ref, qer = bswgen.assemble(items)
    want = pairs.copy()
    oracle.get_scores(_oparams(), want, ref, qer, w, nthreads=8)
    got = pairs.copy()
    e.get_scores(got, ref, qer, w)
    _assert_same(want, got, f"gq32 255/256 w={w}")
    e.close()


def test_group_kernel_32lane_golden(golden):
    """Every golden batch through the 32-lane form where the scoring qualifies (BSW_OPT_GQ32_MAX)."""
    engines, ran = {}, 0
    for name, pairs, ref, qer, w, sc in golden:
        key = tuple(sorted(sc.items()))
        if key not in engines:
            engines[key] = bsw.Engine(_gparams(sc), gq32_max=1_000_000)
        got = pairs.copy()
        for f in bsw.OUT_FIELDS:
            got[f] = -9
        engines[key].get_scores(got, ref, qer, w)
        _assert_same(pairs, got, f"gq32 golden {name}")
        ran += engines[key].last_stats().n_group
    assert ran > 0
    for e in engines.values():
        e.close()
