"""Seeds -> chains (include/bsw_fmi.h bsw_mem_chain_device; bwa's mem_chain + mem_chain_flt) and
the whole GPU front end of mem_align1_core: SMEM seeding -> SA -> chains -> mem_chain2aln.

CPU: C1 regenerates the reference's own data (tests/golden/c1_fingerprint.json, written by
tests/golden/make_c1_fingerprint.py against benchmark_threading.sh:42-70); the C oracle
(oracle/chain_ref.c) equals an independent Python transcription (tests/memchain_py.py) on a
repetitive reference with sampled repeats; the oracle pipeline aligns every C1 read end to end.
GPU: the product's chaining and the whole pipeline equal the oracle.  Parity vs upstream is
unpinned (no upstream source or fixtures for this step)."""

import json
import os

import numpy as np
import pytest

import bsw
import c1data
import hiprt
import memchain_py
import oracle
from conftest import ROOT
from test_fmi import repetitive_ref, sample_reads


def dispersed_copies_ref(n=200_000, copies=60, L=300, seed=2):
    """random reference with `copies` dispersed copies of one L-bp element, a few carrying 1-3
    substitutions: a read of the element has one chain per copy (tens of chains, many of equal
    weight), which drives mem_chain_flt's introsort past its insertion-sort cutoff"""
    rng = np.random.default_rng(seed)
    ref = rng.integers(0, 4, n, dtype=np.uint8)
    elem = rng.integers(0, 4, L, dtype=np.uint8)
    for c in range(copies):
        a = 1000 + c * ((n - 2000) // copies)
        e = elem.copy()
        if c % 3 == 1:
            k = rng.integers(0, L, int(rng.integers(1, 4)))
            e[k] = (e[k] + 1) % 4
        ref[a:a + L] = e if c % 2 == 0 else (3 - e[::-1])
    reads = np.stack([elem[o:o + 151] for o in rng.integers(0, L - 151, 80)]).astype(np.uint8)
    return ref, reads.reshape(-1), np.arange(80, dtype=np.int64) * 151, np.full(80, 151, np.int32)


def _two_strand(ref):
    return np.concatenate([ref, (3 - ref[::-1])]).astype(np.uint8)


def _copt_dict(o):
    return {f: getattr(o, f) for f, _ in o._fields_}


@pytest.fixture(scope="module")
def c1():
    return c1data.workload()


def test_c1_is_the_reference_generators_data(c1):
    ref, reads, off, lens, starts = c1
    fp = json.load(open(os.path.join(ROOT, "tests", "golden", "c1_fingerprint.json")))
    mine = c1data.fingerprint(ref, starts)
    for k in ("ref_sha256", "starts_sha256", "ref_head", "first_starts"):
        assert mine[k] == fp[k], k
    assert len(ref) == 1_000_000 and len(lens) == 10_000 and np.all(lens == 150)
    assert np.array_equal(reads[:150], ref[starts[0]:starts[0] + 150])


def _oracle_front(ref, reads, off, lens, cap=64, copt=None):
    f = oracle.FmiRef(ref)
    mems, cnt = f.collect_intv(reads, off, lens, cap=cap, nthreads=8)
    seeds, sr, sc = oracle.mem_chain(f.sa(), len(ref), lens, mems, cnt, copt)
    return f, mems, cnt, seeds, sr, sc


def test_c1_oracle_pipeline_aligns_every_read_end_to_end(c1):
    ref, reads, off, lens, starts = c1
    f, mems, cnt, seeds, sr, sc = _oracle_front(ref, reads, off, lens)
    out, ext = oracle.chain2aln(oracle.make_params(), bsw.ext_opt(l_pac=len(ref)), _two_strand(ref), reads, off, lens,
                                seeds, sr, sc)
    first = np.r_[True, sr[1:] != sr[:-1]]               # each read's first chain's first seed ...
    assert np.array_equal(np.unique(sr), np.arange(10_000))
    best = np.zeros(10_000, np.int64) - 1
    for k in np.flatnonzero(ext):
        if out["truesc"][k] == 150:
            best[sr[k]] = k
    assert np.all(best >= 0), "every read has an extended 150-bp end-to-end region"
    b = out[best]
    assert np.all(b["qb"] == 0) and np.all(b["qe"] == 150) and np.all(b["rb"] == starts) and \
        np.all(b["re"] == starts + 150)
    assert np.all(sc[first] == 0)


def _chain_lists(seeds, sr, sc, n):
    out = [[] for _ in range(n)]
    for k in range(len(seeds)):
        r, c = int(sr[k]), int(sc[k])
        while len(out[r]) <= c:
            out[r].append([])
        out[r][c].append((int(seeds[k]["rbeg"]), int(seeds[k]["qbeg"]), int(seeds[k]["len"])))
    return out


@pytest.mark.parametrize("max_occ", [500, 3])
def test_oracle_chaining_equals_python_transcription(max_occ):
    """repetitive reference (duplications, inverted copy, tandem repeats, near copies): many
    chains per read; max_occ 3 samples the repeat intervals with a step; both strands"""
    ref = repetitive_ref(60_000, seed=4)
    reads, off, lens = sample_reads(ref, 300, 151, seed=9)
    copt = oracle.chain_opt(max_occ=max_occ)
    f, mems, cnt, seeds, sr, sc = _oracle_front(ref, reads, off, lens, cap=2048, copt=copt)
    assert np.all(cnt <= 2048)
    got = _chain_lists(seeds, sr, sc, len(lens))
    sa = f.sa()
    opt = _copt_dict(copt)
    many = 0
    for r in range(len(lens)):
        ms = [(int(m["k"]), int(m["l"]), int(m["s"]), int(m["info"])) for m in mems[r, :cnt[r]]]
        want = memchain_py.mem_chain_read(opt, sa, len(ref), int(lens[r]), ms)
        assert got[r] == want, r
        many += len(want) > 1
    assert many > 20, "the sample must hold reads with several chains"


def test_oracle_chaining_many_chains_equals_python():
    """tens of chains per read (dispersed copies): the weight sort runs klib's partitioning
    introsort, not only its insertion sort; C oracle == Python transcription chain for chain"""
    ref, reads, off, lens = dispersed_copies_ref()
    copt = oracle.chain_opt()
    f, mems, cnt, seeds, sr, sc = _oracle_front(ref, reads, off, lens, cap=2048, copt=copt)
    got = _chain_lists(seeds, sr, sc, len(lens))
    sa = f.sa()
    for r in range(len(lens)):
        ms = [(int(m["k"]), int(m["l"]), int(m["s"]), int(m["info"])) for m in mems[r, :cnt[r]]]
        assert got[r] == memchain_py.mem_chain_read(_copt_dict(copt), sa, len(ref), int(lens[r]), ms), r
    assert max(len(c) for c in got) > 40


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_chaining_many_chains_equals_oracle():
    ref, reads, off, lens = dispersed_copies_ref()
    f, mems, cnt, wseeds, wsr, wsc = _oracle_front(ref, reads, off, lens, cap=2048)
    fmi = bsw.Fmi(ref)
    d_reads = hiprt.DeviceBuffer.from_array(reads)
    (seeds, sr, sc), _, _ = bsw.seed_and_chain(fmi, d_reads, off, lens, cap=2048)
    assert np.array_equal(sr, wsr) and np.array_equal(sc, wsc)
    for fld in ("rbeg", "qbeg", "len"):
        assert np.array_equal(seeds[fld], wseeds[fld]), fld
    assert sc.max() > 40
    fmi.close()


@pytest.mark.gpu
def test_c1_gpu_seeding_chaining_extension_equal_oracle(c1):
    """C1 (the reference's own 10K exact reads vs its 1 Mb reference) through the GPU front end:
    SMEM seeding -> SA -> chains -> mem_chain2aln on the resident two-strand text; seeds,
    chains and every region equal the oracle, and every read aligns end to end (truesc 150)."""
    ref, reads, off, lens, starts = c1
    f, mems, cnt, wseeds, wsr, wsc = _oracle_front(ref, reads, off, lens)
    fmi = bsw.Fmi(ref)
    d_reads = hiprt.DeviceBuffer.from_array(reads)
    (seeds, sr, sc), (d_seeds, d_sr, d_sc), (d_off, d_len) = bsw.seed_and_chain(fmi, d_reads, off, lens, cap=64)
    assert np.array_equal(sr, wsr) and np.array_equal(sc, wsc)
    for fld in ("rbeg", "qbeg", "len"):
        assert np.array_equal(seeds[fld], wseeds[fld]), fld
    T = _two_strand(ref)
    opt = bsw.ext_opt(l_pac=len(ref))
    want, wext = oracle.chain2aln(oracle.make_params(), opt, T, reads, off, lens, wseeds, wsr, wsc)
    eng = bsw.Engine()
    bsw.set_reference(eng, T)
    ns = len(seeds)
    d_out = hiprt.DeviceBuffer(ns * bsw.ALNREG_DTYPE.itemsize)
    d_ext = hiprt.DeviceBuffer(ns * 4)
    bsw.chain2aln_resident(eng, d_reads.ptr, d_off.ptr, d_len.ptr, len(lens), d_seeds.ptr, d_sr.ptr, d_sc.ptr, ns,
                           d_out.ptr, d_ext.ptr, opt)
    got = d_out.download(np.zeros(ns, dtype=bsw.ALNREG_DTYPE))
    gext = d_ext.download(np.zeros(ns, dtype=np.int32))
    assert np.array_equal(gext, wext)
    for fld in bsw.ALNREG_DTYPE.names:
        assert np.array_equal(got[fld], want[fld]), fld
    full = (gext == 1) & (got["truesc"] == 150)
    assert np.array_equal(np.unique(sr[full]), np.arange(10_000))
    eng.close()
    fmi.close()


@pytest.mark.gpu
@pytest.mark.parametrize("max_occ", [500, 3])
def test_gpu_chaining_equals_oracle_repetitive(max_occ):
    """repetitive 2 Mb reference, 20K reads from both strands with errors / N / random reads:
    bsw_mem_chain_device == oracle_mem_chain; a seed_cap below the need is BSW_E_RANGE with the
    needed count"""
    ref = repetitive_ref(2_000_000, seed=21)
    reads, off, lens = sample_reads(ref, 20_000, 151, seed=5)
    copt_o = oracle.chain_opt(max_occ=max_occ)
    f, mems, cnt, wseeds, wsr, wsc = _oracle_front(ref, reads, off, lens, cap=1024, copt=copt_o)
    fmi = bsw.Fmi(ref)
    d_reads = hiprt.DeviceBuffer.from_array(reads)
    copt = bsw.chain_opt(max_occ=max_occ)
    (seeds, sr, sc), _, (d_off, d_len) = bsw.seed_and_chain(fmi, d_reads, off, lens, cap=1024, copt=copt)
    assert len(seeds) == len(wseeds)
    assert np.array_equal(sr, wsr) and np.array_equal(sc, wsc)
    for fld in ("rbeg", "qbeg", "len"):
        assert np.array_equal(seeds[fld], wseeds[fld]), fld
    assert np.bincount(sc).size > 2
    # too small a seed_cap: BSW_E_RANGE and the count needed
    d_mems = hiprt.DeviceBuffer(len(lens) * 1024 * bsw.BWTINTV_DTYPE.itemsize)
    d_cnt = hiprt.DeviceBuffer(len(lens) * 4)
    assert fmi.collect_intv_device(d_reads.ptr, d_off.ptr, d_len.ptr, len(lens), 151, d_mems.ptr, 1024, d_cnt.ptr) == 0
    small = hiprt.DeviceBuffer(16 * 10)
    rc, need = fmi.mem_chain_device(d_len.ptr, len(lens), d_mems.ptr, 1024, d_cnt.ptr, small.ptr, small.ptr,
                                    small.ptr, 10, copt)
    assert rc == -34 and need == len(wseeds)
    fmi.close()


@pytest.mark.gpu
def test_gpu_front_end_pe_reads_equal_oracle():
    """4 Mb reference with repeat copies, 40K reads from both strands (1% substitutions, N,
    random reads): GPU seeding -> chains -> mem_chain2aln (resident two-strand text, l_pac
    clamp) == the oracle pipeline, region for region"""
    import bench
    ref = bench.seeding_reference(4_000_000, seed=3)
    reads, off, lens = bench.seeding_reads(ref, 40_000, 151, seed=8)
    f, mems, cnt, wseeds, wsr, wsc = _oracle_front(ref, reads, off, lens, cap=256)
    T = _two_strand(ref)
    opt = bsw.ext_opt(l_pac=len(ref))
    want, wext = oracle.chain2aln(oracle.make_params(), opt, T, reads, off, lens, wseeds, wsr, wsc)
    fmi = bsw.Fmi(ref)
    d_reads = hiprt.DeviceBuffer.from_array(reads)
    (seeds, sr, sc), (d_seeds, d_sr, d_sc), (d_off, d_len) = bsw.seed_and_chain(fmi, d_reads, off, lens, cap=256)
    assert np.array_equal(sr, wsr) and np.array_equal(sc, wsc) and np.array_equal(seeds["rbeg"], wseeds["rbeg"])
    eng = bsw.Engine()
    bsw.set_reference(eng, T)
    ns = len(seeds)
    d_out = hiprt.DeviceBuffer(ns * bsw.ALNREG_DTYPE.itemsize)
    d_ext = hiprt.DeviceBuffer(ns * 4)
    bsw.chain2aln_resident(eng, d_reads.ptr, d_off.ptr, d_len.ptr, len(lens), d_seeds.ptr, d_sr.ptr, d_sc.ptr, ns,
                           d_out.ptr, d_ext.ptr, opt)
    got = d_out.download(np.zeros(ns, dtype=bsw.ALNREG_DTYPE))
    gext = d_ext.download(np.zeros(ns, dtype=np.int32))
    assert np.array_equal(gext, wext)
    for fld in bsw.ALNREG_DTYPE.names:
        assert np.array_equal(got[fld], want[fld]), fld
    assert (seeds["rbeg"] >= len(ref)).mean() > 0.3          # reverse-strand seeds took part
    eng.close()
    fmi.close()
