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
