"""Recovery of host-buffer calls from engine errors (bsw.h, bsw_get_scores):
a device run that fails with BSW_E_NOMEM / BSW_E_HIP is rerun -- on its device after the cached
slots are freed, on the context's other devices, then in halves -- before any error reaches the
caller.  Failures are injected with the test-only BSW_OPT_TEST_FAIL_ALLOC (the next k device
buffer growths fail as out of memory, process-wide).  Every recovered call must give the oracle's
outputs; only when every step fails does the call return BSW_E_NOMEM (and then the shim exits,
upstream's convention).  Reference plan: PHASE2_IMPLEMENTATION_SUMMARY.md:210-225."""

import numpy as np
import pytest

import bsw
import bswgen
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def batch():
    pairs, ref, qer = bsw.synth_batch(200_000)
    want = pairs.copy()
    oracle.get_scores(oracle.make_params(), want, ref, qer, 100, nthreads=16)
    return pairs, ref, qer, want


def _same(want, got, tag):
    for f in bsw.OUT_FIELDS:
        bad = int((want[f] != got[f]).sum())
        assert bad == 0, f"{tag}: field {f} differs in {bad} pairs"
    for f in ("idr", "idq", "id", "len1", "len2", "h0", "seqid", "regid"):
        assert np.array_equal(want[f], got[f]), f"{tag}: input field {f} changed"


def _run(e, pairs, ref, qer, fail):
    got = pairs.copy()
    e.set_option("test_fail_alloc", fail)
    try:
        e.get_scores(got, ref, qer, 100)
    finally:
        e.set_option("test_fail_alloc", 0)
    return got, e.last_stats()


@pytest.mark.parametrize("n", [200_000, 50_000, 3000])
def test_recovery_retry_on_fresh_slot(batch, n):
    """one injected failure: the first run fails, the rerun after freeing the cached slots works
    (n = 3000: the coalesced small-call path; 50K: one chunk; 200K: the chunked pipeline)"""
    pairs, ref, qer, want = batch
    e = bsw.Engine()
    got, st = _run(e, pairs[:n], ref, qer, 1)
    _same(want[:n], got, f"retry n={n}")
    assert st.recovery == 1
    got, st = _run(e, pairs[:n], ref, qer, 0)        # and the engine works on afterwards
    _same(want[:n], got, f"after retry n={n}")
    assert st.recovery == 0
    e.close()


def test_recovery_in_halves(batch):
    """two injected failures on a one-device context: the first run and the rerun fail, the call
    completes in halves (a one-chunk call, <= 128K pairs: each run stops at its first failed
    allocation, so the two failures are exactly those two runs)"""
    pairs, ref, qer, want = batch
    e = bsw.Engine()
    got, st = _run(e, pairs[:100_000], ref, qer, 2)
    _same(want[:100_000], got, "halves")
    assert st.recovery == 3
    e.close()


def test_recovery_on_another_device(batch):
    """two logical devices on the box's GPU (bsw_create_on, the rehearsal of a 2-GPU context): a
    call small enough to run whole on one device fails there twice and completes on the other"""
    pairs, ref, qer, want = batch
    e = bsw.Engine(devices=[0, 0])
    got, st = _run(e, pairs[:60_000], ref, qer, 2)
    _same(want[:60_000], got, "other device")
    assert st.recovery == 2
    # a split call (>= BSW_OPT_SPLIT_MIN pairs): one device's range fails and is recovered
    got, st = _run(e, pairs, ref, qer, 1)
    _same(want, got, "split call")
    assert st.recovery in (1, 2) and st.n_devices == 2
    e.close()


def test_recovery_exhausted_returns_nomem(batch):
    """every allocation fails: the call returns BSW_E_NOMEM (the caller's records keep their input
    fields), and the engine recovers fully once allocations work again"""
    pairs, ref, qer, want = batch
    e = bsw.Engine()
    got = pairs[:20_000].copy()
    e.set_option("test_fail_alloc", 1_000_000)
    try:
        with pytest.raises(bsw.BswError, match="-12"):
            e.get_scores(got, ref, qer, 100)
    finally:
        e.set_option("test_fail_alloc", 0)
    for f in ("idr", "idq", "len1", "len2", "h0"):
        assert np.array_equal(got[f], pairs[:20_000][f])
    got, st = _run(e, pairs[:20_000], ref, qer, 0)
    _same(want[:20_000], got, "after exhaustion")
    e.close()


def test_recovery_random_shapes():
    """mixed shapes (long queries, int16-unsafe h0: several kernel classes) recovered in halves"""
    pairs, ref, qer = bswgen.random_pairs(12_000, seed=77, qlen=(0, 400), tlen=(0, 500), h0=(0, 32700))
    want = pairs.copy()
    oracle.get_scores(oracle.make_params(), want, ref, qer, 100, nthreads=8)
    e = bsw.Engine()
    got, st = _run(e, pairs, ref, qer, 2)
    _same(want, got, "random shapes")
    assert st.recovery == 3
    e.close()


def test_fail_alloc_option_range():
    e = bsw.Engine()
    for bad in (-1, 1_000_001):
        with pytest.raises(bsw.BswError):
            e.set_option("test_fail_alloc", bad)
    e.set_option("test_fail_alloc", 0)
    e.close()
