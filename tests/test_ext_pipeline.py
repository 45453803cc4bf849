"""Seed-extension pipeline (include/bsw_ext.h): job builder + result
interpreter around the batch engine.

CPU tests pin the pipeline oracle (oracle/ext_ref.c, C) against an independent Python
transcription of the same upstream consumer (mem_chain2aln's extension half) built on the
Python ksw_extend2, plus geometric properties on synthetic reads.  GPU tests require the
engine's bsw_extend_seeds to equal the oracle read for read.  Parity unpinned by the
reference (no upstream fixtures for this step)."""

import numpy as np
import pytest

import bsw
import oracle
from ksw_ext_ref import ksw_extend2 as py_ksw_extend2


def _workload(n, seed=11, ref_len=200_000, **kw):
    ref = bsw.synth_reference(ref_len, seed=seed)
    reads, off, lens, seeds, origin = bsw.synth_reads(ref, n, cfg=bsw.reads_cfg(seed=seed, **kw))
    return ref, reads, off, lens, seeds, origin


def _cal_max_gap(p, a, w, qlen):
    l_del = int((qlen * a - p.o_del) / p.e_del + 1.0)
    l_ins = int((qlen * a - p.o_ins) / p.e_ins + 1.0)
    return min(max(max(l_del, l_ins), 1), w << 1)


def py_chain_window(p, opt, ref_len, l_query, chain):
    """mem_chain2aln's rmax[] (bwa src/bwamem.c): min / max of the chain's seeds' reach, clipped
    to the text, and on a two-strand text (opt.l_pac > 0) the first seed's side of l_pac."""
    a = p.mat[0]
    lo, hi = ref_len, 0
    for s in chain:
        qbeg, rbeg, slen = int(s["qbeg"]), int(s["rbeg"]), int(s["len"])
        lo = min(lo, rbeg - (qbeg + _cal_max_gap(p, a, opt.w, qbeg)))
        qe = qbeg + slen
        hi = max(hi, rbeg + slen + (l_query - qe) + _cal_max_gap(p, a, opt.w, l_query - qe))
    lo, hi = max(lo, 0), min(hi, ref_len)
    if opt.l_pac > 0 and lo < opt.l_pac < hi:
        if int(chain[0]["rbeg"]) < opt.l_pac:
            hi = opt.l_pac
        else:
            lo = opt.l_pac
    return lo, hi


def py_extend(p, opt, ref, reads, off, lens, seeds, windows=None):
    """Independent transcription of the extension half of mem_chain2aln, one seed per read
    (windows[i] = the chain's target window; default: the seed's own, a chain of one)."""
    a = p.mat[0]
    mat = list(p.mat)
    out = np.zeros(len(seeds), dtype=bsw.ALNREG_DTYPE)
    for i, s in enumerate(seeds):
        if s["len"] <= 0:
            continue
        q = reads[off[i]:off[i] + lens[i]]
        l_query, qbeg, rbeg, slen = int(lens[i]), int(s["qbeg"]), int(s["rbeg"]), int(s["len"])
        rmax0, rmax1 = windows[i] if windows is not None else py_chain_window(p, opt, len(ref), l_query, [s])
        qe = qbeg + slen
        r = out[i]
        aw = [opt.w, opt.w]
        r["seedlen0"] = slen
        score = -1                                        # a->score before the first band try
        if qbeg:
            qs = q[:qbeg][::-1]
            rs = ref[rmax0:rbeg][::-1]
            for t in range(opt.max_band_try):
                prev = score
                aw[0] = opt.w << t
                score, qle, tle, gtle, gscore, max_off = py_ksw_extend2(
                    list(qs), list(rs), mat, p.o_del, p.e_del, p.o_ins, p.e_ins, aw[0], opt.pen_clip5,
                    p.zdrop, slen * a)
                if score == prev or max_off < (aw[0] >> 1) + (aw[0] >> 2):
                    break
            if gscore <= 0 or gscore <= score - opt.pen_clip5:
                r["qb"], r["rb"], r["truesc"] = qbeg - qle, rbeg - tle, score
            else:
                r["qb"], r["rb"], r["truesc"] = 0, rbeg - gtle, gscore
        else:
            score = slen * a
            r["truesc"], r["qb"], r["rb"] = score, 0, rbeg
        if qe != l_query:
            sc0 = score
            re = rbeg + slen
            for t in range(opt.max_band_try):
                prev = score
                aw[1] = opt.w << t
                score, qle, tle, gtle, gscore, max_off = py_ksw_extend2(
                    list(q[qe:]), list(ref[re:rmax1]), mat, p.o_del, p.e_del, p.o_ins, p.e_ins, aw[1],
                    opt.pen_clip3, p.zdrop, sc0)
                if score == prev or max_off < (aw[1] >> 1) + (aw[1] >> 2):
                    break
            if gscore <= 0 or gscore <= score - opt.pen_clip3:
                r["qe"], r["re"] = qe + qle, re + tle
                r["truesc"] += score - sc0
            else:
                r["qe"], r["re"] = l_query, re + gtle
                r["truesc"] += gscore - sc0
        else:
            r["qe"], r["re"] = l_query, rbeg + slen
        r["score"] = score
        r["w"] = max(aw)
    return out


def _same(want, got, tag):
    bad = np.zeros(len(want), bool)
    for f in bsw.ALNREG_DTYPE.names:
        bad |= want[f] != got[f]
    if bad.any():
        i = int(np.flatnonzero(bad)[0])
        raise AssertionError(f"{tag}: {int(bad.sum())}/{len(want)} reads differ; first {i}: "
                             f"want {want[i]} got {got[i]}")


def test_reads_generator_seeds_are_exact():
    ref, reads, off, lens, seeds, origin = _workload(3000)
    ok = seeds["len"] > 0
    assert ok.mean() > 0.95
    for i in np.flatnonzero(ok)[:500]:
        s = seeds[i]
        q = reads[off[i] + s["qbeg"]: off[i] + s["qbeg"] + s["len"]]
        assert np.array_equal(q, ref[s["rbeg"]: s["rbeg"] + s["len"]])
        assert s["len"] >= 19


@pytest.mark.parametrize("w,try_,clip", [(100, 2, (5, 5)), (8, 2, (5, 5)), (20, 1, (0, 100)), (3, 3, (2, 9))])
def test_oracle_pipeline_c_equals_python(w, try_, clip):
    ref, reads, off, lens, seeds, _ = _workload(150, seed=3 + w, ref_len=50_000, p_sub=0.04, p_indel=0.01)
    p = oracle.make_params()
    opt = bsw.ExtOpt(w=w, pen_clip5=clip[0], pen_clip3=clip[1], max_band_try=try_)
    want = py_extend(p, opt, ref, reads, off, lens, seeds)
    got = oracle.extend_seeds(p, opt, ref, reads, off, lens, seeds)
    _same(want, got, f"C vs Python w={w}")


def test_oracle_pipeline_geometry():
    ref, reads, off, lens, seeds, origin = _workload(2000, seed=5, p_unrelated=0.0)
    p = oracle.make_params()
    reg = oracle.extend_seeds(p, bsw.ext_opt(), ref, reads, off, lens, seeds)
    ok = seeds["len"] > 0
    r, s = reg[ok], seeds[ok]
    assert np.all(r["qb"] <= s["qbeg"]) and np.all(r["qe"] >= s["qbeg"] + s["len"])
    assert np.all(r["rb"] <= s["rbeg"]) and np.all(r["re"] >= s["rbeg"] + s["len"])
    # related reads at 2% substitutions mostly align end to end at their true origin
    full = (r["qb"] == 0) & (r["qe"] == lens[ok])
    assert full.mean() > 0.9
    assert np.mean(np.abs(r["rb"][full] - origin[ok][full]) <= 3) > 0.95
    assert np.all(r["truesc"] <= r["qe"] - r["qb"])        # a = 1


def test_exact_reads_full_length():
    ref, reads, off, lens, seeds, origin = _workload(300, seed=9, p_sub=0.0, p_indel=0.0, p_unrelated=0.0)
    reg = oracle.extend_seeds(oracle.make_params(), bsw.ext_opt(), ref, reads, off, lens, seeds)
    ok = seeds["len"] > 0
    assert np.all(reg["qb"][ok] == 0) and np.all(reg["qe"][ok] == 150)
    assert np.all(reg["rb"][ok] == origin[ok]) and np.all(reg["re"][ok] == origin[ok] + 150)
    nn = ok & np.array([not np.any(ref[o:o + 150] == 4) for o in origin])
    assert np.all(reg["truesc"][nn] == 150)


# ---------------------------------------------------------------- GPU: engine == oracle
@pytest.mark.gpu
@pytest.mark.parametrize("w,try_,clip", [(100, 2, (5, 5)), (10, 2, (5, 5)), (20, 1, (0, 100)),
                                          (3, 3, (2, 9))])
def test_gpu_pipeline_matches_oracle(w, try_, clip):
    ref, reads, off, lens, seeds, _ = _workload(20_000, seed=21 + w, ref_len=2_000_000, p_sub=0.03,
                                               p_indel=0.005)
    opt = bsw.ExtOpt(w=w, pen_clip5=clip[0], pen_clip3=clip[1], max_band_try=try_)
    want = oracle.extend_seeds(oracle.make_params(), opt, ref, reads, off, lens, seeds)
    eng = bsw.Engine()
    got = bsw.extend_seeds(eng, ref, reads, off, lens, seeds, opt)
    _same(want, got, f"GPU pipeline w={w}")
    st = bsw.ext_last_stats(eng)
    assert st.n_pairs[0] > 0 and st.n_pairs[2] > 0
    if try_ > 1 and w <= 10:
        assert st.n_pairs[1] + st.n_pairs[3] > 0       # band retries exercised
    eng.close()


@pytest.mark.gpu
def test_gpu_pipeline_edges():
    """Seeds at read/reference ends, reads without seeds, N-rich reference."""
    ref = bsw.synth_reference(5000, seed=2, p_n=0.05)
    reads, off, lens, seeds, origin = bsw.synth_reads(ref, 2000, cfg=bsw.reads_cfg(seed=4, read_len=120))
    seeds[::7]["len"] = 0                                     # no seed
    seeds[1::7]["qbeg"] = 0                                   # seed at the read start
    seeds[2::7]["qbeg"] = lens[2::7] - seeds[2::7]["len"]     # seed at the read end
    for i in range(3, len(seeds), 7):                         # seed at the reference start
        seeds[i]["rbeg"], seeds[i]["qbeg"], seeds[i]["len"] = 0, 10, 19
    opt = bsw.ext_opt()
    want = oracle.extend_seeds(oracle.make_params(), opt, ref, reads, off, lens, seeds)
    eng = bsw.Engine()
    got = bsw.extend_seeds(eng, ref, reads, off, lens, seeds, opt)
    _same(want, got, "GPU pipeline edges")
    eng.close()


# ---------------------------------------------------------------- GPU: device-resident pipeline
@pytest.mark.gpu
@pytest.mark.parametrize("w,try_,clip", [(100, 2, (5, 5)), (10, 2, (5, 5)), (20, 1, (0, 100)),
                                          (3, 3, (2, 9))])
def test_gpu_device_pipeline_matches_oracle(w, try_, clip):
    """bsw_extend_seeds_device (job build / retries / interpretation on the GPU, resident
    reference) == the CPU restatement == the host-built pipeline."""
    ref, reads, off, lens, seeds, _ = _workload(20_000, seed=21 + w, ref_len=2_000_000, p_sub=0.03,
                                               p_indel=0.005)
    opt = bsw.ExtOpt(w=w, pen_clip5=clip[0], pen_clip3=clip[1], max_band_try=try_)
    want = oracle.extend_seeds(oracle.make_params(), opt, ref, reads, off, lens, seeds)
    eng = bsw.Engine()
    bsw.set_reference(eng, ref)
    got = bsw.extend_seeds_resident(eng, reads, off, lens, seeds, opt)
    _same(want, got, f"device pipeline w={w}")
    st = bsw.ext_last_stats(eng)
    assert st.n_pairs[0] > 0 and st.n_pairs[2] > 0
    if try_ > 1 and w <= 10:
        assert st.n_pairs[1] + st.n_pairs[3] > 0
    _same(bsw.extend_seeds(eng, ref, reads, off, lens, seeds, opt), got, "host vs device pipeline")
    eng.close()


@pytest.mark.gpu
def test_gpu_device_pipeline_edges():
    """Seeds at read/reference ends, reads without seeds, N-rich reference, varying read
    lengths; no resident reference -> BSW_E_INVAL; bad seed -> BSW_E_RANGE."""
    ref = bsw.synth_reference(5000, seed=2, p_n=0.05)
    reads, off, lens, seeds, origin = bsw.synth_reads(ref, 2000, cfg=bsw.reads_cfg(seed=4, read_len=120))
    seeds[::7]["len"] = 0
    seeds[1::7]["qbeg"] = 0
    seeds[2::7]["qbeg"] = lens[2::7] - seeds[2::7]["len"]
    for i in range(3, len(seeds), 7):
        seeds[i]["rbeg"], seeds[i]["qbeg"], seeds[i]["len"] = 0, 10, 19
    lens = lens.copy()
    lens[5::11] = np.maximum(seeds[5::11]["qbeg"] + seeds[5::11]["len"], lens[5::11] - 30)   # shorter reads
    opt = bsw.ext_opt()
    want = oracle.extend_seeds(oracle.make_params(), opt, ref, reads, off, lens, seeds)
    eng = bsw.Engine()
    with pytest.raises(bsw.BswError):
        bsw.extend_seeds_resident(eng, reads, off, lens, seeds, opt)        # no resident reference
    bsw.set_reference(eng, ref)
    got = bsw.extend_seeds_resident(eng, reads, off, lens, seeds, opt)
    _same(want, got, "device pipeline edges")
    bad = seeds.copy()
    bad[0]["rbeg"] = len(ref)
    bad[0]["len"] = 5
    with pytest.raises(bsw.BswError):
        bsw.extend_seeds_resident(eng, reads, off, lens, bad, opt)
    eng.close()


@pytest.mark.gpu
def test_gpu_pipelines_chunked():
    """Calls split into read chunks (the int32 SeqPair-offset guard that applies above ~3.9M reads,
    forced small by BSW_OPT_EXT_CHUNK) give the unsplit results on both pipeline forms."""
    ref, reads, off, lens, seeds, _ = _workload(5_000, seed=5, ref_len=500_000, p_sub=0.03, p_indel=0.005)
    opt = bsw.ext_opt()
    want = oracle.extend_seeds(oracle.make_params(), opt, ref, reads, off, lens, seeds)
    eng = bsw.Engine(ext_chunk=1234)
    host = bsw.extend_seeds(eng, ref, reads, off, lens, seeds, opt)
    st = bsw.ext_last_stats(eng)
    assert st.n_pairs[0] > 0 and st.n_pairs[2] > 0                 # aggregated over the chunks
    bsw.set_reference(eng, ref)
    dev = bsw.extend_seeds_resident(eng, reads, off, lens, seeds, opt)
    _same(want, host, "host-built pipeline, chunked")
    _same(want, dev, "device pipeline, chunked")
    eng.close()


@pytest.mark.gpu
def test_gpu_pipelines_no_fork():
    """Class launches run serially on the caller's stream (BSW_OPT_FORK = 0) give the forked
    results on both pipeline forms."""
    ref, reads, off, lens, seeds, _ = _workload(3_000, seed=6, ref_len=400_000, p_sub=0.03, p_indel=0.005)
    opt = bsw.ext_opt()
    want = oracle.extend_seeds(oracle.make_params(), opt, ref, reads, off, lens, seeds)
    eng = bsw.Engine(fork=0)
    host = bsw.extend_seeds(eng, ref, reads, off, lens, seeds, opt)
    bsw.set_reference(eng, ref)
    dev = bsw.extend_seeds_resident(eng, reads, off, lens, seeds, opt)
    _same(want, host, "host-built pipeline, no fork")
    _same(want, dev, "device pipeline, no fork")
    eng.close()


@pytest.mark.gpu
def test_host_and_device_pipelines_accept_the_same_reads():
    """Both forms validate per read (the device form used to reject a whole batch when the
    longest read + 2w + 1 passed BSW_MAX_LEN): a 32,700-base read whose windows fit is accepted
    by both and equals the oracle; a read whose LEFT window passes BSW_MAX_LEN is rejected by
    both; a seed across l_pac of a two-strand text is rejected by both."""
    ref = bsw.synth_reference(200_000, seed=8)
    ref[ref == 4] = 1
    L = 32_700
    reads = np.concatenate([ref[1000:1000 + L], ref[50_000:50_150]]).astype(np.uint8)
    off = np.array([0, L], np.int64)
    lens = np.array([L, 150], np.int32)
    seeds = np.zeros(2, dtype=bsw.SEED_DTYPE)
    seeds[0]["rbeg"], seeds[0]["qbeg"], seeds[0]["len"] = 1000 + 16_000, 16_000, 40
    seeds[1]["rbeg"], seeds[1]["qbeg"], seeds[1]["len"] = 50_020, 20, 30
    opt = bsw.ext_opt()
    want = oracle.extend_seeds(oracle.make_params(), opt, ref, reads, off, lens, seeds)
    eng = bsw.Engine()
    bsw.set_reference(eng, ref)
    _same(want, bsw.extend_seeds(eng, ref, reads, off, lens, seeds, opt), "host, long read")
    _same(want, bsw.extend_seeds_resident(eng, reads, off, lens, seeds, opt), "device, long read")
    bad = seeds.copy()
    bad[0]["qbeg"], bad[0]["rbeg"], bad[0]["len"] = L - 20, 1000 + L - 20, 20   # LEFT window > BSW_MAX_LEN
    for f in (lambda: bsw.extend_seeds(eng, ref, reads, off, lens, bad, opt),
              lambda: bsw.extend_seeds_resident(eng, reads, off, lens, bad, opt)):
        with pytest.raises(bsw.BswError):
            f()
    T = np.concatenate([ref, np.where(ref < 4, 3 - ref, ref)[::-1]]).astype(np.uint8)
    opt2 = bsw.ext_opt(l_pac=len(ref))
    cross = seeds[1:].copy()
    cross[0]["rbeg"], cross[0]["qbeg"], cross[0]["len"] = len(ref) - 10, 20, 30
    bsw.set_reference(eng, T)
    for f in (lambda: bsw.extend_seeds(eng, T, reads, off[1:], lens[1:], cross, opt2),
              lambda: bsw.extend_seeds_resident(eng, reads, off[1:], lens[1:], cross, opt2)):
        with pytest.raises(bsw.BswError):
            f()
    eng.close()
