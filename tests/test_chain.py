"""mem_chain2aln over chains (include/bsw_ext.h bsw_chain2aln): upstream's
per-read chain / seed order with contained-seed skipping, batched across reads in rounds.

CPU: the oracle's literal restatement (oracle/ext_ref.c oracle_chain2aln) on the paired-end,
several-seeds-per-read generator (bsw_synth_pe_seeds) -- single-seed chains reduce to the plain
extension, skipped seeds lie inside an earlier region of their read, seeds are exact.
GPU: the engine's round-batched forms (host reads / resident reads) == the oracle."""

import numpy as np
import pytest

import bsw
import hiprt
import oracle

REF_LEN = 4_000_000


@pytest.fixture(scope="module")
def ref():
    return bsw.synth_reference(REF_LEN, seed=11)


def test_generator_seeds_exact_and_paired(ref):
    reads, off, lens, seeds, sr, sc = bsw.synth_pe_seeds(ref, 3000)
    q = reads.reshape(-1, 150)
    assert len(off) == 6000 and np.all(np.diff(sr) >= 0)
    for k in range(len(seeds)):
        s = seeds[k]
        assert np.array_equal(q[sr[k], s["qbeg"]:s["qbeg"] + s["len"]], ref[s["rbeg"]:s["rbeg"] + s["len"]])
    per_read = np.bincount(sr, minlength=6000)
    assert per_read.mean() > 1.5 and per_read.max() <= 9
    assert set(np.unique(sc)) <= {0, 1} and (sc == 1).any()


def test_single_seed_chains_equal_plain_extension(ref):
    reads, off, lens, seeds, sr, sc = bsw.synth_pe_seeds(ref, 1500)
    first = np.r_[True, sr[1:] != sr[:-1]]            # one (the longest) seed per read
    s1, r1 = seeds[first], sr[first]
    P, opt = oracle.make_params(), bsw.ext_opt()
    want = oracle.extend_seeds(P, opt, ref, reads, off[r1], lens[r1], s1)
    got, ext = oracle.chain2aln(P, opt, ref, reads, off, lens, s1, r1, np.zeros(len(s1), np.int32))
    assert ext.all()
    for f in bsw.ALNREG_DTYPE.names:
        assert np.array_equal(got[f], want[f]), f


def test_skipped_seeds_are_inside_an_earlier_region(ref):
    reads, off, lens, seeds, sr, sc = bsw.synth_pe_seeds(ref, 2000)
    out, ext = oracle.chain2aln(oracle.make_params(), bsw.ext_opt(), ref, reads, off, lens, seeds, sr, sc)
    skipped = np.flatnonzero(ext == 0)
    assert 0.2 * len(seeds) < len(skipped) < len(seeds)
    for k in skipped:
        s = seeds[k]
        mates = np.flatnonzero((sr == sr[k]) & (ext == 1))
        assert any(out[m]["rb"] <= s["rbeg"] and s["rbeg"] + s["len"] <= out[m]["re"] and
                   out[m]["qb"] <= s["qbeg"] and s["qbeg"] + s["len"] <= out[m]["qe"] for m in mates), k
        assert out[k]["re"] == 0 and out[k]["w"] == 0


def _same(want, got, tag):
    for f in bsw.ALNREG_DTYPE.names:
        bad = np.flatnonzero(want[f] != got[f])
        assert len(bad) == 0, f"{tag}: {f} differs at {len(bad)} seeds, first {bad[:5]}"


@pytest.mark.gpu
def test_chain2aln_host_equals_oracle(ref):
    reads, off, lens, seeds, sr, sc = bsw.synth_pe_seeds(ref, 20000, pair_base=77)
    opt = bsw.ext_opt()
    want, wext = oracle.chain2aln(oracle.make_params(), opt, ref, reads, off, lens, seeds, sr, sc)
    eng = bsw.Engine()
    got, gext = bsw.chain2aln(eng, ref, reads, off, lens, seeds, sr, sc, opt)
    assert np.array_equal(wext, gext)
    _same(want, got, "chain2aln host")
    st = bsw.chain_last_stats(eng)
    assert st.rounds >= 2 and st.n_skipped == int((gext == 0).sum()) and st.n_extended == int(gext.sum())
    eng.close()


@pytest.mark.gpu
def test_chain2aln_device_200k_reads_equal_oracle(ref):
    """>= 200K paired-end reads (100K fragments) through the resident-reads form."""
    reads, off, lens, seeds, sr, sc = bsw.synth_pe_seeds(ref, 100_000, pair_base=5000)
    opt = bsw.ext_opt()
    want, wext = oracle.chain2aln(oracle.make_params(), opt, ref, reads, off, lens, seeds, sr, sc)
    eng = bsw.Engine()
    bsw.set_reference(eng, ref)
    d_reads = hiprt.DeviceBuffer.from_array(reads)
    got, gext = bsw.chain2aln_device(eng, d_reads.ptr, off, lens, seeds, sr, sc, opt)
    assert np.array_equal(wext, gext)
    _same(want, got, "chain2aln device 200K reads")
    eng.close()


@pytest.mark.gpu
def test_chain2aln_resident_equals_oracle(ref):
    """every array device-resident (bsw_chain2aln_resident: chain order, containment and picks on
    the GPU) == the oracle; an unsorted seed_read is rejected"""
    reads, off, lens, seeds, sr, sc = bsw.synth_pe_seeds(ref, 30_000, pair_base=9000)
    opt = bsw.ext_opt()
    want, wext = oracle.chain2aln(oracle.make_params(), opt, ref, reads, off, lens, seeds, sr, sc)
    eng = bsw.Engine()
    bsw.set_reference(eng, ref)
    d = {k: hiprt.DeviceBuffer.from_array(v) for k, v in
         dict(reads=reads, off=off, lens=lens, seeds=seeds, sr=sr, sc=sc).items()}
    d_out = hiprt.DeviceBuffer(len(seeds) * bsw.ALNREG_DTYPE.itemsize)
    d_ext = hiprt.DeviceBuffer(len(seeds) * 4)
    bsw.chain2aln_resident(eng, d["reads"].ptr, d["off"].ptr, d["lens"].ptr, len(lens), d["seeds"].ptr, d["sr"].ptr,
                           d["sc"].ptr, len(seeds), d_out.ptr, d_ext.ptr, opt)
    got = d_out.download(np.zeros(len(seeds), dtype=bsw.ALNREG_DTYPE))
    gext = d_ext.download(np.zeros(len(seeds), dtype=np.int32))
    assert np.array_equal(wext, gext)
    _same(want, got, "chain2aln resident")
    st = bsw.chain_last_stats(eng)
    assert st.rounds >= 2 and st.n_extended == int(gext.sum())
    bad = hiprt.DeviceBuffer.from_array(sr[::-1].copy())
    with pytest.raises(bsw.BswError):
        bsw.chain2aln_resident(eng, d["reads"].ptr, d["off"].ptr, d["lens"].ptr, len(lens), d["seeds"].ptr, bad.ptr,
                               d["sc"].ptr, len(seeds), d_out.ptr, d_ext.ptr, opt)
    eng.close()


# ---------------------------------------------------------------- the chain's target window
# mem_chain2aln takes ONE target window per chain (rmax[]: min / max over the chain's seeds, and on
# bwa's forward + reverse-complement text the first seed's side of l_pac); every seed of the chain
# extends inside it.  Checked against the independent Python transcription (test_ext_pipeline).

def revcomp(codes):
    c = np.asarray(codes, dtype=np.uint8)
    return np.where(c < 4, 3 - c, c)[::-1].astype(np.uint8)


def _chains(sr, sc):
    """[(start, end)) runs of equal (read, chain)"""
    cut = np.flatnonzero(np.r_[True, (sr[1:] != sr[:-1]) | (sc[1:] != sc[:-1]), True])
    return list(zip(cut[:-1], cut[1:]))


def test_chain_window_spans_every_seed_of_the_chain(ref):
    from test_ext_pipeline import py_chain_window, py_extend
    reads, off, lens, seeds, sr, sc = bsw.synth_pe_seeds(ref, 3000, pair_base=31)
    P, opt = oracle.make_params(), bsw.ext_opt()
    out, ext = oracle.chain2aln(P, opt, ref, reads, off, lens, seeds, sr, sc)
    picked, wins, differ = [], [], 0
    for a, b in _chains(sr, sc):
        if b - a < 2:
            continue
        win = py_chain_window(P, opt, len(ref), int(lens[sr[a]]), seeds[a:b])
        for k in range(a, b):
            if ext[k]:
                own = py_chain_window(P, opt, len(ref), int(lens[sr[k]]), seeds[k:k + 1])
                differ += own != win
                picked.append(k)
                wins.append(win)
        if len(picked) >= 120:
            break
    assert differ >= 20, "the sample must hold seeds whose own window differs from the chain's"
    k = np.array(picked)
    want = py_extend(P, opt, ref, reads, off[sr[k]], lens[sr[k]], seeds[k], windows=wins)
    _same(want, out[k], "oracle chain2aln vs Python with chain windows")


def _two_strand_boundary_case(ref_len=60_000, seed=5):
    """bwa's two-strand text T = ref + revcomp(ref) (l_pac = ref_len) and reads whose chain
    windows cross l_pac from either side: forward reads ending 0..40 bases before l_pac (their
    right reach runs past it) and reverse-strand reads starting 0..40 bases after it."""
    ref = bsw.synth_reference(ref_len, seed=seed)
    ref[ref == 4] = 0
    T = np.concatenate([ref, revcomp(ref)])
    rng = np.random.default_rng(seed)
    L, reads, off, lens, seeds, sr, sc = 150, [], [], [], [], [], []
    for i in range(64):
        fwd = i % 2 == 0
        gap = int(rng.integers(0, 41))
        start = ref_len - L + 60 - gap if fwd else ref_len + gap - 60
        start = min(max(start, 0), 2 * ref_len - L)
        r = T[start:start + L].copy()
        mut = rng.random(L) < 0.03
        r[mut] = (r[mut] + rng.integers(1, 4, mut.sum())) % 4
        # one or two seeds inside the read on the read's own strand side of l_pac
        qb = int(rng.integers(0, 20))
        for j, (q0, ln) in enumerate(((qb, 25), (qb + 40, 22))):
            rb = start + q0
            if (rb < ref_len) != (start + q0 + ln <= ref_len) or (fwd and rb + ln > ref_len) or \
                    (not fwd and rb < ref_len):
                continue
            r[q0:q0 + ln] = T[rb:rb + ln]
            seeds.append((rb, q0, ln)); sr.append(i); sc.append(0)
        off.append(i * L); lens.append(L); reads.append(r)
    seeds = np.array(seeds, dtype=[("rbeg", "<i8"), ("qbeg", "<i4"), ("len", "<i4")]).view(bsw.SEED_DTYPE)
    return (T, ref_len, np.concatenate(reads), np.array(off, np.int64), np.array(lens, np.int32), seeds,
            np.array(sr, np.int32), np.array(sc, np.int32))


def test_chain_window_keeps_the_first_seeds_strand():
    from test_ext_pipeline import py_chain_window, py_extend
    T, l_pac, reads, off, lens, seeds, sr, sc = _two_strand_boundary_case()
    P = oracle.make_params()
    opt = bsw.ext_opt(l_pac=l_pac)
    out, ext = oracle.chain2aln(P, opt, T, reads, off, lens, seeds, sr, sc)
    crossing = 0
    wins = {}
    for a, b in _chains(sr, sc):
        win = py_chain_window(P, opt, len(T), int(lens[sr[a]]), seeds[a:b])
        raw = py_chain_window(P, bsw.ext_opt(), len(T), int(lens[sr[a]]), seeds[a:b])
        crossing += raw != win
        for k in range(a, b):
            wins[k] = win
    assert crossing >= 40, "most chains must have windows that cross l_pac"
    k = np.flatnonzero(ext)
    want = py_extend(P, opt, T, reads, off[sr[k]], lens[sr[k]], seeds[k], windows=[wins[i] for i in k])
    _same(want, out[k], "strand-clamped chain windows")
    fwd = seeds["rbeg"][k] < l_pac
    assert np.all(out["re"][k][fwd] <= l_pac) and np.all(out["rb"][k][~fwd] >= l_pac)


@pytest.mark.gpu
def test_chain_windows_on_gpu_equal_oracle(ref):
    """multi-seed chains (one window per chain) and the l_pac strand clamp through the host,
    device and resident chain2aln forms; a seed across l_pac is rejected by every form"""
    T, l_pac, reads, off, lens, seeds, sr, sc = _two_strand_boundary_case()
    P = oracle.make_params()
    eng = bsw.Engine()
    cases = [(T, bsw.ext_opt(l_pac=l_pac), reads, off, lens, seeds, sr, sc, "boundary")]
    r2, o2, l2, s2, sr2, sc2 = bsw.synth_pe_seeds(ref, 20000, pair_base=4242)
    cases.append((ref, bsw.ext_opt(), r2, o2, l2, s2, sr2, sc2, "pe chains"))
    for (R, opt, rd, of, ln, sd, rr, cc, tag) in cases:
        want, wext = oracle.chain2aln(P, opt, R, rd, of, ln, sd, rr, cc)
        got, gext = bsw.chain2aln(eng, R, rd, of, ln, sd, rr, cc, opt)
        assert np.array_equal(wext, gext)
        _same(want, got, f"{tag} host")
        bsw.set_reference(eng, R)
        d_reads = hiprt.DeviceBuffer.from_array(rd)
        got, gext = bsw.chain2aln_device(eng, d_reads.ptr, of, ln, sd, rr, cc, opt)
        assert np.array_equal(wext, gext)
        _same(want, got, f"{tag} device")
    bad = seeds.copy()
    bad[0]["rbeg"], bad[0]["qbeg"], bad[0]["len"] = l_pac - 10, 0, 20
    opt = bsw.ext_opt(l_pac=l_pac)
    with pytest.raises(bsw.BswError):
        bsw.chain2aln(eng, T, reads, off, lens, bad, sr, sc, opt)
    bsw.set_reference(eng, T)
    d_reads = hiprt.DeviceBuffer.from_array(reads)
    with pytest.raises(bsw.BswError):
        bsw.chain2aln_device(eng, d_reads.ptr, off, lens, bad, sr, sc, opt)
    eng.close()
