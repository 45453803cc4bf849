"""FM-index SMEM seeding (include/bsw_fmi.h).

CPU: the oracle (oracle/fmi_ref.c: bwt_smem1a / bwt_seed_strategy1 / mem_collect_intv restated)
is pinned by brute force -- every interval's occurrence count, SA row and reverse-complement row
against naive string search over T = ref + revcomp(ref); the pass-1 SMEMs are exactly the
super-maximal exact matches of the read (computed naively); the product's host-built suffix
array / BWT / counts equal the oracle's.  Parity vs upstream itself is unpinned (the reference
holds no source or fixtures for this path).
GPU: bsw_mem_collect_intv(_device) == oracle on random, repetitive and edge-case inputs.
"""
import bisect
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import oracle  # noqa: E402
import bsw  # noqa: E402

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def repetitive_ref(n, seed):
    """random reference with segment duplications, an inverted copy and tandem repeats"""
    rng = np.random.default_rng(seed)
    ref = rng.integers(0, 4, n, dtype=np.uint8)
    seg = n // 10
    ref[2 * seg:3 * seg] = ref[seg // 2:seg // 2 + seg]                          # duplication
    ref[4 * seg:4 * seg + seg // 2] = 3 - ref[seg:seg + seg // 2][::-1]          # inverted copy
    ref[6 * seg:6 * seg + 120] = np.tile(np.array([0, 1, 1], np.uint8), 40)      # tandem repeat
    ref[7 * seg:7 * seg + 60] = 2                                                # homopolymer
    for k in range(8):                                                           # 8 near copies
        a = 8 * seg + k * (seg // 8)
        ref[a:a + 40] = ref[5 * seg:5 * seg + 40]
        ref[a + 20] = (ref[a + 20] + 1 + k % 3) % 4
    return ref


def sample_reads(ref, n, L, seed, p_sub=0.02, p_n=0.002, p_rand=0.1, p_rc=0.5):
    """reads from either strand with substitutions / N, plus random reads: (reads, off, len)"""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        if rng.random() < p_rand:
            r = rng.integers(0, 4, L, dtype=np.uint8)
        else:
            p = int(rng.integers(0, len(ref) - L))
            r = ref[p:p + L].copy()
            if rng.random() < p_rc:
                r = (3 - r[::-1]).astype(np.uint8)
            m = rng.random(L) < p_sub
            r[m] = (r[m] + rng.integers(1, 4, int(m.sum()))) % 4
        r[rng.random(L) < p_n] = 4
        out.append(r.astype(np.uint8))
    lens = np.array([len(r) for r in out], dtype=np.int32)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    return np.concatenate(out) if out else np.zeros(1, np.uint8), off, lens


class Naive:
    """brute-force string view of T$ = ref + revcomp(ref) + '$'"""

    def __init__(self, ref):
        t = np.concatenate([ref, 3 - ref[::-1]]).astype(np.uint8)
        self.T = ACGT[t].tobytes().decode()
        self.n = len(self.T)
        # '$' sorts before every base: suffix strings with '#' (< 'A') appended
        self.sorted = sorted(self.T[i:] + "#" for i in range(self.n + 1))

    def count(self, p):
        c, i = 0, self.T.find(p)
        while i >= 0:
            c += 1
            i = self.T.find(p, i + 1)
        return c

    def first_row(self, p):
        return bisect.bisect_left(self.sorted, p)


def s_of(read):
    return ACGT[np.minimum(read, 3)].tobytes().decode()


def revcomp(p):
    return p[::-1].translate(str.maketrans("ACGT", "TGCA"))


@pytest.fixture(scope="module")
def small_world():
    ref = repetitive_ref(3000, 5)
    return ref, oracle.FmiRef(ref), Naive(ref)


def test_oracle_index_matches_naive(small_world):
    ref, o, nv = small_world
    sa = o.sa()
    assert [nv.T[i:] + "#" for i in sa] == nv.sorted
    bwt = o.bwt()
    assert bwt[o.sentinel] == 4 and sa[o.sentinel] == 0
    assert list(o.count) == [1] + list(1 + np.cumsum([nv.T.count(c) for c in "ACGT"]))


def test_oracle_intervals_pinned_by_brute_force(small_world):
    ref, o, nv = small_world
    reads, off, lens = sample_reads(ref, 60, 100, 11)
    out, cnt = o.collect_intv(reads, off, lens, cap=256, opt=oracle.mem_opt(min_seed_len=12))
    checked = 0
    for i in range(len(lens)):
        rd = reads[off[i]:off[i] + lens[i]]
        prev = None
        for v in out[i, :cnt[i]]:
            m, e = int(v["info"] >> 32), int(v["info"] & 0xffffffff)
            assert 0 <= m < e <= lens[i] and (rd[m:e] < 4).all()
            p = s_of(rd[m:e])
            assert int(v["s"]) == nv.count(p), (i, m, e)
            assert int(v["k"]) == nv.first_row(p)
            assert int(v["l"]) == nv.first_row(revcomp(p))
            key = (int(v["info"]), int(v["k"]), int(v["s"]), int(v["l"]))
            assert prev is None or prev <= key                     # sorted by info, then k, s, l
            prev = key
            checked += 1
    assert checked > 200


def naive_smems(nv, rd):
    """super-maximal exact matches of the read: [m, e) occurring in T, not extendable left or
    right, not contained in another such match (bases 4 never match)"""
    L = len(rd)
    ends = []
    for m in range(L):
        e = m
        while e < L and rd[e] < 4 and nv.count(s_of(rd[m:e + 1])) > 0:
            e += 1
        ends.append(e)
    mems = {(m, ends[m]) for m in range(L) if ends[m] > m and (m == 0 or ends[m - 1] < ends[m])}
    return {(m, e) for (m, e) in mems if not any(a <= m and e <= b and (a, b) != (m, e) for (a, b) in mems)}


def test_oracle_pass1_is_the_smem_set(small_world):
    ref, o, nv = small_world
    reads, off, lens = sample_reads(ref, 40, 60, 12, p_sub=0.04)
    only_pass1 = oracle.mem_opt(min_seed_len=1, max_mem_intv=0, split_factor=1000.0)
    out, cnt = o.collect_intv(reads, off, lens, cap=256, opt=only_pass1)
    for i in range(len(lens)):
        rd = reads[off[i]:off[i] + lens[i]]
        got = {(int(v["info"] >> 32), int(v["info"] & 0xffffffff)) for v in out[i, :cnt[i]]}
        assert got == naive_smems(nv, rd), i


def test_oracle_passes_2_and_3_fire(small_world):
    """the repetitive reference makes re-seeding (pass 2) and LAST-like seeds (pass 3) add
    intervals that pass 1 alone does not produce"""
    ref, o, nv = small_world
    seg = len(ref) // 10
    reads = np.concatenate([ref[seg // 2 + 10:seg // 2 + 110], ref[8 * seg:8 * seg + 100], ref[5 * seg:5 * seg + 100]])
    off = np.array([0, 100, 200], dtype=np.int64)
    lens = np.array([100, 100, 100], dtype=np.int32)
    _, c_all = o.collect_intv(reads, off, lens, opt=oracle.mem_opt())
    _, c_1 = o.collect_intv(reads, off, lens, opt=oracle.mem_opt(max_mem_intv=0, split_factor=1000.0))
    _, c_12 = o.collect_intv(reads, off, lens, opt=oracle.mem_opt(max_mem_intv=0))
    assert (c_12 >= c_1).all() and (c_all >= c_12).all()
    assert c_12.sum() > c_1.sum() and c_all.sum() > c_12.sum()


@pytest.mark.parametrize("seed,n,L,msl", [(5, 3000, 100, 12), (7, 20000, 151, 19), (9, 60000, 151, 12)])
def test_tied_intervals_are_identical(seed, n, L, msl):
    """mem_collect_intv sorts intervals by info = qbeg << 32 | qend with klib's ks_introsort,
    which leaves ties in an implementation order; here ties are ordered by (k, s, l).  That is no
    parity gap: equal info means the same read substring, whose SA interval (k, s) and
    reverse-complement row l are unique, so tied records are identical and every order of them
    is the same sequence -- checked on repetitive references where ties do occur (pass-3
    LAST-like seeds repeating a pass-1 / pass-2 span)."""
    ref = repetitive_ref(n, seed)
    o = oracle.FmiRef(ref)
    reads, off, lens = sample_reads(ref, 400, L, seed + 1, p_sub=0.03)
    out, cnt = o.collect_intv(reads, off, lens, cap=512, opt=oracle.mem_opt(min_seed_len=msl))
    ties = 0
    for i in range(len(lens)):
        v = out[i, :cnt[i]]
        same = v["info"][1:] == v["info"][:-1]
        ties += int(same.sum())
        for f in ("k", "l", "s"):
            assert np.array_equal(v[f][1:][same], v[f][:-1][same]), (i, f)
    assert ties > 0


@pytest.mark.parametrize("seed,n", [(1, 5000), (3, 40000)])
def test_host_builder_equals_oracle(seed, n):
    """the product's prefix-doubling suffix array / BWT / counts (host-only index, no GPU) ==
    the oracle's comparison-sorted ones"""
    ref = repetitive_ref(n, seed)
    o = oracle.FmiRef(ref)
    f = bsw.Fmi(ref, device=-1)
    info = f.info()
    assert info.n == o.n and info.sentinel == o.sentinel and list(info.count) == list(o.count)
    assert np.array_equal(f.sa(), o.sa())
    assert np.array_equal(f.bwt(), o.bwt())
    f.close()


def test_host_builder_rejects_bad_input():
    with pytest.raises(bsw.BswError):
        bsw.Fmi(np.array([0, 1, 4, 2], dtype=np.uint8), device=-1)
    f = bsw.Fmi(np.array([0], dtype=np.uint8), device=-1)          # tiny reference
    assert list(f.sa()) == [2, 0, 1] and f.info().count[4] == 3
    f.close()


# ------------------------------------------------------------------------------------- GPU

def _compare(o_out, o_cnt, g_out, g_cnt):
    assert np.array_equal(o_cnt, g_cnt)
    for i in range(len(o_cnt)):
        c = min(int(o_cnt[i]), o_out.shape[1])
        assert np.array_equal(o_out[i, :c], g_out[i, :c]), i


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [None, bsw.FMI_NO_TEXT], ids=["text_mode", "blocks_only"])
@pytest.mark.parametrize("kind,n_ref,n_reads,L", [("random", 200_000, 4000, 151), ("repetitive", 100_000, 3000, 151),
                                                  ("repetitive", 50_000, 500, 250)])
def test_gpu_collect_intv_equals_oracle(kind, n_ref, n_reads, L, flags):
    """GPU mem_collect_intv == the oracle, with the text-mode walk (single-occurrence intervals
    extended by comparing read and text, BSW_FMI_NO_TEXT off) and with occurrence blocks only."""
    ref = repetitive_ref(n_ref, 9) if kind == "repetitive" else np.random.default_rng(9).integers(0, 4, n_ref, dtype=np.uint8)
    reads, off, lens = sample_reads(ref, n_reads, L, 21)
    o = oracle.FmiRef(ref)
    f = bsw.Fmi(ref, flags=flags)
    for opt in (dict(), dict(min_seed_len=15), dict(max_mem_intv=0), dict(split_width=50, min_seed_len=11)):
        o_out, o_cnt = o.collect_intv(reads, off, lens, cap=320, opt=oracle.mem_opt(**opt), nthreads=8)
        g_out, g_cnt = f.collect_intv(reads, off, lens, cap=320, opt=bsw.mem_opt(**opt))
        _compare(o_out, o_cnt, g_out, g_cnt)
    f.close()


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [None, bsw.FMI_NO_TEXT], ids=["text_mode", "blocks_only"])
def test_gpu_collect_intv_edges(flags):
    ref = repetitive_ref(20_000, 4)
    o = oracle.FmiRef(ref)
    f = bsw.Fmi(ref, flags=flags)
    seg = len(ref) // 10
    rd = [np.zeros(0, np.uint8), np.array([2], np.uint8), np.full(30, 4, np.uint8),
          np.concatenate([[4], ref[100:160], [4]]).astype(np.uint8), ref[7 * seg - 10:7 * seg + 90].copy(),
          ref[6 * seg:6 * seg + 150].copy(), (3 - ref[200:350][::-1]).astype(np.uint8), ref[:80].copy(),
          ref[-80:].copy(), np.full(100, 2, np.uint8)]
    lens = np.array([len(r) for r in rd], dtype=np.int32)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    reads = np.concatenate(rd).astype(np.uint8)
    o_out, o_cnt = o.collect_intv(reads, off, lens, cap=2048)
    g_out, g_cnt = f.collect_intv(reads, off, lens, cap=2048)
    _compare(o_out, o_cnt, g_out, g_cnt)
    assert g_cnt[0] == 0 and g_cnt[2] == 0 and g_cnt[-1] > 1000      # 100 G vs a 60-G run: 1572
    # too small a cap: the call reports BSW_E_RANGE, reads that fit are exact, the others are
    # flagged with a count > cap (a lower bound: re-seeding only sees the stored SMEMs)
    with pytest.raises(bsw.BswError):
        f.collect_intv(reads, off, lens, cap=2)
    g2, c2 = f.collect_intv(reads, off, lens, cap=2, strict=False)
    fit = o_cnt <= 2
    assert np.array_equal(c2[fit], o_cnt[fit]) and (c2[~fit] > 2).all() and (c2[~fit] <= o_cnt[~fit]).all()
    for i in np.nonzero(fit)[0]:
        assert np.array_equal(g2[i, :o_cnt[i]], o_out[i, :o_cnt[i]])
    f.close()


@pytest.mark.gpu
@pytest.mark.parametrize("levels", [0, 1, 5, 12])
@pytest.mark.parametrize("flags", [None, bsw.FMI_GPU_BUILD | bsw.FMI_WIDE], ids=["narrow", "wide"])
def test_gpu_kmer_table_depths_equal_oracle(levels, flags, monkeypatch):
    """The k-mer interval table (BSW_FMI_KTAB levels; 0 = off, 12 = far past log4 |T| on this
    reference, so most deep entries are empty intervals) serves the short strings of every walk:
    pass-1 / pass-2 forward, the backward sweeps, the re-seeding bound, pass 3.  Outputs == the
    oracle at every depth, narrow and wide, with long runs and an N-rich read set."""
    monkeypatch.setenv("BSW_FMI_KTAB", str(levels))
    ref = _long_runs_ref(60_000, 11)
    reads, off, lens = sample_reads(ref, 2500, 151, 13, p_n=0.01)
    o = oracle.FmiRef(ref)
    f = bsw.Fmi(ref, flags=flags)
    for opt in (dict(), dict(min_seed_len=11, split_width=50), dict(max_mem_intv=0)):
        o_out, o_cnt = o.collect_intv(reads, off, lens, cap=512, opt=oracle.mem_opt(**opt), nthreads=8)
        g_out, g_cnt = f.collect_intv(reads, off, lens, cap=512, opt=bsw.mem_opt(**opt))
        _compare(o_out, o_cnt, g_out, g_cnt)
    f.close()


@pytest.mark.gpu
@pytest.mark.parametrize("wide_ent", [None, "1"], ids=["packed16", "plain32"])
def test_gpu_wide_entry_forms_equal_oracle(wide_ent):
    """The wide index's interval vectors in packed 16-B entries (default: 40-bit k / l, 32-bit s,
    15-bit ends + the text flag) and in plain 32-B entries (BSW_FMI_PLAIN_ENT): == the oracle."""
    ref = _long_runs_ref(80_000, 17)
    reads, off, lens = sample_reads(ref, 2000, 151, 19, p_n=0.01)
    o = oracle.FmiRef(ref)
    f = bsw.Fmi(ref, flags=bsw.FMI_GPU_BUILD | bsw.FMI_WIDE | (bsw.FMI_PLAIN_ENT if wide_ent else 0))
    for opt in (dict(), dict(min_seed_len=11, split_width=50)):
        o_out, o_cnt = o.collect_intv(reads, off, lens, cap=512, opt=oracle.mem_opt(**opt), nthreads=8)
        g_out, g_cnt = f.collect_intv(reads, off, lens, cap=512, opt=bsw.mem_opt(**opt))
        _compare(o_out, o_cnt, g_out, g_cnt)
    f.close()


@pytest.mark.gpu
def test_gpu_device_api_and_sa_lookup():
    import hiprt
    ref = np.random.default_rng(6).integers(0, 4, 100_000, dtype=np.uint8)
    reads, off, lens = sample_reads(ref, 2000, 151, 8)
    o = oracle.FmiRef(ref)
    f = bsw.Fmi(ref)
    cap = 128
    d_reads, d_off, d_len = (hiprt.DeviceBuffer.from_array(a) for a in (reads, off, lens))
    d_mems = hiprt.DeviceBuffer(len(lens) * cap * 32)
    d_cnt = hiprt.DeviceBuffer(len(lens) * 4)
    assert f.collect_intv_device(d_reads.ptr, d_off.ptr, d_len.ptr, len(lens), 151, d_mems.ptr, cap, d_cnt.ptr) == 0
    g_out = d_mems.download(np.zeros((len(lens), cap), dtype=bsw.BWTINTV_DTYPE))
    g_cnt = d_cnt.download(np.zeros(len(lens), dtype=np.int32))
    o_out, o_cnt = o.collect_intv(reads, off, lens, cap=cap, nthreads=8)
    _compare(o_out, o_cnt, g_out, g_cnt)
    # bwt_sa over every row an interval starts at, plus out-of-range rows
    ks = np.concatenate([o_out[i, :o_cnt[i]]["k"] for i in range(len(lens))] + [np.array([o.n + 1, 2**40], np.uint64)])
    d_k = hiprt.DeviceBuffer.from_array(ks.astype(np.uint64))
    d_pos = hiprt.DeviceBuffer(len(ks) * 8)
    f.sa_device(d_k.ptr, len(ks), d_pos.ptr)
    pos = d_pos.download(np.zeros(len(ks), dtype=np.int64))
    sa = o.sa()
    assert np.array_equal(pos[:-2], sa[ks[:-2].astype(np.int64)]) and (pos[-2:] == -1).all()
    f.close()


# --------------------------------------------------------------- GPU-built and wide (64-bit) indexes

def _long_runs_ref(n, seed):
    """repetitive_ref plus a 400-base homopolymer and a 600-base dinucleotide repeat: tie groups of
    hundreds of suffixes equal on 27 bases (the builder's host-sorted path)"""
    ref = repetitive_ref(n, seed)
    ref[n // 3:n // 3 + 400] = 1
    ref[n // 2:n // 2 + 600] = np.tile(np.array([0, 3], np.uint8), 300)
    return ref


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["repetitive", "random", "long_runs"])
@pytest.mark.parametrize("flags", [bsw.FMI_GPU_BUILD, bsw.FMI_GPU_BUILD | bsw.FMI_WIDE])
def test_gpu_builder_equals_host_builder(kind, flags):
    """bsw_fmi_build2 on the GPU (bucketed radix sort of 27-base keys, tie groups by comparison),
    narrow and wide (64-bit) layouts: suffix array, BWT, sentinel and counts == the host
    prefix-doubling builder's"""
    n = 300_000
    ref = {"repetitive": lambda: repetitive_ref(n, 2), "long_runs": lambda: _long_runs_ref(n, 3),
           "random": lambda: np.random.default_rng(5).integers(0, 4, n, dtype=np.uint8)}[kind]()
    h = bsw.Fmi(ref, device=-1)
    g = bsw.Fmi(ref, flags=flags)
    hi, gi = h.info(), g.info()
    assert gi.n == hi.n and gi.sentinel == hi.sentinel and list(gi.count) == list(hi.count)
    assert np.array_equal(g.sa(), h.sa())
    assert np.array_equal(g.bwt(), h.bwt())
    h.close()
    g.close()


@pytest.mark.gpu
def test_wide_index_seeding_and_chaining_equal_oracle():
    """the wide layout (64-bit rows, counts and suffix array -- what a 3 Gb two-strand genome
    needs) runs mem_collect_intv, bwt_sa and mem_chain exactly like the narrow one: == oracle"""
    import hiprt
    ref = _long_runs_ref(200_000, 7)
    reads, off, lens = sample_reads(ref, 3000, 151, 13)
    o = oracle.FmiRef(ref)
    f = bsw.Fmi(ref, flags=bsw.FMI_GPU_BUILD | bsw.FMI_WIDE)
    for opt in (dict(), dict(min_seed_len=15), dict(split_width=50, min_seed_len=11)):
        o_out, o_cnt = o.collect_intv(reads, off, lens, cap=2048, opt=oracle.mem_opt(**opt), nthreads=8)
        g_out, g_cnt = f.collect_intv(reads, off, lens, cap=2048, opt=bsw.mem_opt(**opt))
        _compare(o_out, o_cnt, g_out, g_cnt)
    o_out, o_cnt = o.collect_intv(reads, off, lens, cap=2048, nthreads=8)
    ks = np.concatenate([o_out[i, :o_cnt[i]]["k"] for i in range(len(lens))] + [np.array([o.n + 1], np.uint64)])
    d_k = hiprt.DeviceBuffer.from_array(ks.astype(np.uint64))
    d_pos = hiprt.DeviceBuffer(len(ks) * 8)
    f.sa_device(d_k.ptr, len(ks), d_pos.ptr)
    pos = d_pos.download(np.zeros(len(ks), dtype=np.int64))
    assert np.array_equal(pos[:-1], o.sa()[ks[:-1].astype(np.int64)]) and pos[-1] == -1
    seeds, sr, sc = oracle.mem_chain(o.sa(), len(ref), lens, o_out, o_cnt)
    d_reads = hiprt.DeviceBuffer.from_array(reads)
    (gs, gsr, gsc), _, _ = bsw.seed_and_chain(f, d_reads, off, lens, cap=2048)
    assert np.array_equal(gsr, sr) and np.array_equal(gsc, sc) and np.array_equal(gs["rbeg"], seeds["rbeg"])
    f.close()


@pytest.mark.gpu
def test_gpu_builder_at_64mb():
    """bsw_fmi_build's own choice at 64 Mb (GPU builder, narrow) == the wide GPU build, and the
    suffix array is sorted: 20K sampled adjacent rows compared as strings of T$"""
    ref = bsw.synth_reference(64_000_000, seed=7)
    ref[ref > 3] = 2
    a = bsw.Fmi(ref)
    b = bsw.Fmi(ref, flags=bsw.FMI_GPU_BUILD | bsw.FMI_WIDE)
    ia, ib = a.info(), b.info()
    assert ia.n == ib.n == 2 * len(ref) and ia.sentinel == ib.sentinel and list(ia.count) == list(ib.count)
    sa = a.sa()
    assert np.array_equal(sa, b.sa())
    T = np.concatenate([ref, 3 - ref[::-1]]).astype(np.uint8).tobytes()   # '$' = the end: a prefix sorts first
    rng = np.random.default_rng(1)
    for r in rng.integers(0, len(sa) - 1, 20_000):
        x, y = int(sa[r]), int(sa[r + 1])
        u, v = T[x:x + 64], T[y:y + 64]
        assert u < v or (u == v and T[x:] < T[y:]), r
    a.close()
    b.close()


@pytest.mark.gpu
def test_index_self_check():
    """bsw_fmi_check: 0 violations on host-built, GPU-built narrow and wide indexes"""
    ref = _long_runs_ref(120_000, 11)
    for flags in (None, bsw.FMI_GPU_BUILD, bsw.FMI_GPU_BUILD | bsw.FMI_WIDE):
        f = bsw.Fmi(ref, flags=flags)
        assert f.check() == 0, flags
        f.close()


def test_sa_sample_sorted_checker():
    """the host-side sampled suffix-array check of the genome-scale test: 0 on the oracle's suffix
    array of a repetitive reference (long ties walked past the first window), every row sampled;
    a swapped adjacent pair and a duplicated row are found"""
    ref = repetitive_ref(20_000, 5)
    T = np.concatenate([ref, (3 - ref[::-1])]).astype(np.uint8)
    sa = oracle.FmiRef(ref).sa().astype(np.int64)
    n = len(T)
    assert len(sa) == n + 1
    assert _sa_sample_sorted(T, lambda rows: sa[rows], n, 200_000, K=16) == 0
    bad = sa.copy()
    bad[[777, 778]] = bad[[778, 777]]
    assert _sa_sample_sorted(T, lambda rows: bad[rows], n, 200_000, K=16) >= 1
    dup = sa.copy()
    dup[901] = dup[900]
    assert _sa_sample_sorted(T, lambda rows: dup[rows], n, 200_000, K=16) >= 1


@pytest.mark.parametrize("seed,n", [(3, 50_000), (4, 9_000)])
def test_lean_oracle_equals_full(seed, n):
    """the oracle's lean (genome-scale) index -- occurrence checkpoints every 64 rows, SA sampled
    every 32 rows resolved by LF walks (bwa's bwt_sa) -- gives the full form's counts, every SA
    row, the same intervals and the same chains"""
    ref = repetitive_ref(n, seed)
    o = oracle.FmiRef(ref)
    sa = o.sa()
    lean = oracle.FmiRef(ref, sa=sa, lean=True, nthreads=3)
    assert lean.n == o.n and lean.sentinel == o.sentinel and list(lean.count) == list(o.count)
    assert np.array_equal(lean.sa(), sa)
    reads, off, lens = sample_reads(ref, 300, 151, seed + 1)
    a, ca = o.collect_intv(reads, off, lens, cap=512)
    b, cb = lean.collect_intv(reads, off, lens, cap=512, nthreads=2)
    assert np.array_equal(ca, cb) and np.array_equal(a, b)
    for x, y in zip(oracle.mem_chain(sa, len(ref), lens, a, ca), oracle.mem_chain(lean, len(ref), lens, a, ca)):
        assert np.array_equal(x, y)


def _text_check_intervals(T, reads, off, lens, mems, cnt, pos_of, n, max_rows=32):
    """Every interval [k, k + s) (and its reverse-complement rows [l, l + s)) against the text:
    the rows inside (up to max_rows of them) start an exact copy of the read's substring, the two
    rows just outside do not -- so (k, s) and l are exactly the SA ranges of the substring and its
    reverse complement (the SA itself is checked by bsw_fmi_check).  pos_of(rows) -> SA[rows]."""
    rows, want, inside = [], [], []
    for i in range(len(lens)):
        rd = reads[off[i]:off[i] + lens[i]]
        for v in mems[i, :cnt[i]]:
            m, e = int(v["info"] >> 32), int(v["info"] & 0xffffffff)
            p = rd[m:e].tobytes()
            rc = (3 - rd[m:e][::-1]).astype(np.uint8).tobytes()
            k, l, s = int(v["k"]), int(v["l"]), int(v["s"])
            for base, pat in ((k, p), (l, rc)):
                for r in list(range(base, base + min(s, max_rows))):
                    rows.append(r), want.append(pat), inside.append(True)
                for r in (base - 1, base + s):
                    if 0 <= r <= n:
                        rows.append(r), want.append(pat), inside.append(False)
    pos = pos_of(np.array(rows, dtype=np.int64))
    bad = 0
    for r, p, w, ins in zip(rows, pos, want, inside):
        got = T[p:p + len(w)].tobytes() if 0 <= p and p + len(w) <= len(T) else b""
        bad += (got == w) != ins
    return len(rows), bad


def _sa_sample_sorted(T, pos_of, n, m, seed=11, K=64):
    """Rows r, r + 1 for m random r < n: SA[r] and SA[r + 1] (pos_of) must start suffixes of T$ in
    strictly increasing order, compared on the host from the text alone (K-byte windows, ties
    resolved by walking further).  Returns the number of out-of-order pairs (plus bad positions)."""
    r = np.unique(np.random.default_rng(seed).integers(0, n, m))
    p = pos_of(np.concatenate([r, r + 1]))
    pa, pb = p[:len(r)], p[len(r):]
    bad = int(np.sum((pa < 0) | (pa > n) | (pb < 0) | (pb > n) | (pa == pb)))
    L = len(T)

    def win(q, o):
        idx = q[:, None] + o + np.arange(K)[None, :]
        v = T[np.minimum(idx, L - 1)].astype(np.int16)
        v[idx >= L] = -1                                 # '$' and past it: below every base
        return v
    a, b = win(pa, 0), win(pb, 0)
    ne = a != b
    first = np.argmax(ne, axis=1)
    diff = ne.any(axis=1)
    rows = np.arange(len(r))
    bad += int(np.sum(diff & (a[rows, first] > b[rows, first])))
    for i in np.nonzero(~diff)[0]:                       # equal for K bytes: walk on
        o = K
        while True:
            x, y = win(pa[i:i + 1], o)[0], win(pb[i:i + 1], o)[0]
            if (x != y).any():
                j = int(np.argmax(x != y))
                bad += int(x[j] > y[j])
                break
            if pa[i] + o >= L or pb[i] + o >= L:         # both reached '$' together: equal suffixes
                bad += 1
                break
            o += K
    return bad


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_wide_index_at_genome_scale_text_and_oracle():
    """BASELINE C4's index size class inside the GPU suite: a 2.2 Gb reference, whose two-strand
    BWT has 4.4e9 rows (> 2^32: the wide 64-bit layout), built on the GPU and self-checked; 3,000
    mutated PE reads seeded on the GPU with every interval checked against the text at its SA
    rows; chains and mem_chain2aln regions equal to the oracle pipeline run on the product's
    suffix-array rows (the oracle's own index would need ~180 GB at this size)."""
    import bench
    import hiprt
    ref = bench.mem_reference(2200)
    f = bsw.Fmi(ref)
    info = f.info()
    assert info.n + 1 > 2**32
    assert f.check() == 0
    reads, off, lens = bench.pe_reads(ref, 1500, seed=5)
    cap = 256
    mems, cnt = f.collect_intv(reads, off, lens, cap=cap)
    assert (cnt <= cap).all()
    T = np.concatenate([ref, (3 - ref[::-1])]).astype(np.uint8)

    def pos_of(rows):
        d_k = hiprt.DeviceBuffer.from_array(rows.astype(np.uint64))
        d_p = hiprt.DeviceBuffer(len(rows) * 8)
        f.sa_device(d_k.ptr, len(rows), d_p.ptr)
        return d_p.download(np.zeros(len(rows), dtype=np.int64))
    # the suffix array checked on the host, independently of the product's own check: 100K random
    # adjacent rows r, r + 1 hold suffixes of T$ in strictly increasing order ('$' below every base)
    assert _sa_sample_sorted(T, pos_of, info.n, 100_000) == 0
    checked, bad = _text_check_intervals(T, reads, off, lens, mems, cnt, pos_of, info.n)
    assert bad == 0 and checked > 3 * len(lens)
    # chains + regions: the product's GPU pipeline vs the oracle on a compact copy of the SA rows
    # the chains read (interval k -> k', the rows k + t * step laid out at k' + t * step)
    copt = oracle.chain_opt()
    mems_c, src, dst, base = mems.copy(), [], [], 0
    for i in range(len(lens)):
        for t in range(cnt[i]):
            s = int(mems[i, t]["s"])
            step = s // copt.max_occ if s > copt.max_occ else 1
            take = np.arange(0, s, step)[:copt.max_occ]
            mems_c["k"][i, t] = base
            src.append(int(mems[i, t]["k"]) + take)
            dst.append(base + take)
            base += int(take[-1]) + 1 if len(take) else 0
    sa_rows = np.zeros(max(base, 1), dtype=np.int64)
    sa_rows[np.concatenate(dst)] = pos_of(np.concatenate(src))
    seeds, sr, sc = oracle.mem_chain(sa_rows, len(ref), lens, mems_c, cnt, copt)
    d_reads = hiprt.DeviceBuffer.from_array(reads)
    (gs, gsr, gsc), (d_s, d_sr, d_sc), (d_off, d_len) = bsw.seed_and_chain(f, d_reads, off, lens, cap=cap)
    assert np.array_equal(gsr, sr) and np.array_equal(gsc, sc) and np.array_equal(gs, seeds)
    eng = bsw.Engine()
    bsw.set_reference(eng, T)
    opt = bsw.ext_opt(l_pac=len(ref))
    ns = len(seeds)
    d_out, d_ext = hiprt.DeviceBuffer(max(1, ns) * bsw.ALNREG_DTYPE.itemsize), hiprt.DeviceBuffer(max(1, ns) * 4)
    bsw.chain2aln_resident(eng, d_reads.ptr, d_off.ptr, d_len.ptr, len(lens), d_s.ptr, d_sr.ptr, d_sc.ptr, ns,
                           d_out.ptr, d_ext.ptr, opt)
    out = d_out.download(np.zeros(ns, dtype=bsw.ALNREG_DTYPE))
    ext = d_ext.download(np.zeros(ns, dtype=np.int32))
    want, wext = oracle.chain2aln(oracle.make_params(), opt, T, reads, off, lens, seeds, sr, sc, nthreads=8)
    assert np.array_equal(ext, wext)
    for fld in bsw.ALNREG_DTYPE.names:
        assert np.array_equal(out[fld], want[fld]), fld
    eng.close()
    f.close()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpu_builder_satellite_array():
    """A repeat-dense reference for the GPU builder's tie resolution: 100 kb of a
    perfect 171-bp tandem array (alpha-satellite-like) plus 20 kb of a perfect dinucleotide
    repeat inside 2 Mb of random sequence.  Equal 27-base prefixes form ~171 tie groups of ~585
    suffixes whose common prefixes run to the array's end; they are sorted on the host by suffix
    comparison (bsw_fmi_build.hip).  Equal to the host prefix-doubling builder; the build time is
    printed (a perfect multi-Mb array would scale as g log g x array length)."""
    import time
    rng = np.random.default_rng(17)
    ref = rng.integers(0, 4, 2_000_000, dtype=np.uint8)
    unit = rng.integers(0, 4, 171, dtype=np.uint8)
    ref[500_000:600_000] = np.tile(unit, 100_000 // 171 + 1)[:100_000]
    ref[1_200_000:1_220_000] = np.tile(np.array([0, 2], np.uint8), 10_000)
    t = time.perf_counter()
    g = bsw.Fmi(ref, flags=bsw.FMI_GPU_BUILD)
    dt = time.perf_counter() - t
    h = bsw.Fmi(ref, device=-1)
    assert np.array_equal(g.sa(), h.sa())
    assert g.check() == 0
    print(f"GPU build of the 2 Mb satellite reference: {dt:.2f} s")
    assert dt < 120
    g.close()
    h.close()
