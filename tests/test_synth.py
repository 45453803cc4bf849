"""The C2 synthetic workload generator (bwa-mem2-arm_amd/csrc/bsw_synth.c): deterministic,
shaped as BASELINE.json configs[1] says (150 bp query / 300 bp ref, 0.1% N, 10% unrelated
queries, h0 uniform in [19, 100])."""

import numpy as np

import bsw


def test_deterministic_and_seeded():
    a = bsw.synth_batch(2000)
    b = bsw.synth_batch(2000)
    c = bsw.synth_batch(2000, cfg=bsw.synth_cfg(seed=43))
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert not np.array_equal(a[1], c[1])


def test_shape_and_statistics():
    n = 20000
    pairs, ref, qer = bsw.synth_batch(n)
    assert len(ref) == n * 300 and len(qer) == n * 150
    assert np.all(pairs["len1"] == 300) and np.all(pairs["len2"] == 150)
    assert pairs["h0"].min() >= 19 and pairs["h0"].max() <= 100
    assert np.array_equal(pairs["idr"], np.arange(n) * 300)
    assert np.array_equal(pairs["idq"], np.arange(n) * 150)
    assert ref.max() <= 4 and qer.max() <= 4
    n_frac = (ref == 4).mean()
    assert 0.0005 < n_frac < 0.002
    # related queries match their ref prefix at ~98%; unrelated at ~25%
    # (best over small shifts, so an early indel does not make a related query look unrelated)
    Q, R = qer.reshape(n, 150)[:, 10:40], ref.reshape(n, 300)
    ident = np.max([(Q == R[:, 10 + s:40 + s]).mean(axis=1) for s in range(-6, 7)], axis=0)
    unrelated = (ident < 0.6).mean()
    assert 0.08 < unrelated < 0.12


def test_h0_range_option():
    pairs, _, _ = bsw.synth_batch(5000, cfg=bsw.synth_cfg(h0_hi=105))
    assert pairs["h0"].max() == 105
