""".bswb batch files (include/bsw_batch.h): record / replay of
getScores16/8 batches.  CPU: round trip, header checks, corruption detection.  GPU: replay
of a recorded batch reproduces the recorded outputs, and the upstream-compatible shim
records real calls when BSW_RECORD is set."""

import os
import subprocess

import numpy as np
import pytest

import bsw
import bswgen
import oracle
from conftest import ROOT


def _batch_with_outputs(n=800, seed=4):
    pairs, ref, qer = bswgen.random_pairs(n, seed=seed)
    oracle.get_scores(oracle.make_params(), pairs, ref, qer, 100)
    return pairs, ref, qer


def test_round_trip(tmp_path):
    pairs, ref, qer = _batch_with_outputs()
    path = str(tmp_path / "b.bswb")
    p = bsw.default_params(b=3, o_del=5)
    bsw.write_batch(path, pairs, ref, qer, w=77, cell_bits=8, params=p)
    h, p2, r2, q2 = bsw.read_batch(path)
    assert (h.w, h.cell_bits, h.flags, h.n_pairs) == (77, 8, 1, len(pairs))
    assert h.params.o_del == 5 and list(h.params.mat) == list(p.mat)
    assert np.array_equal(p2, pairs) and np.array_equal(r2[:len(ref)], ref) and np.array_equal(q2[:len(qer)], qer)
    assert os.path.getsize(path) == 128 + 56 * len(pairs) + len(ref) + len(qer)


def test_empty_batch(tmp_path):
    path = str(tmp_path / "e.bswb")
    bsw.write_batch(path, np.zeros(0, bsw.SEQPAIR_DTYPE), np.zeros(0, np.uint8), np.zeros(0, np.uint8), w=100,
                    has_outputs=False)
    h, p, _, _ = bsw.read_batch(path)
    assert h.n_pairs == 0 and h.flags == 0 and len(p) == 0


@pytest.mark.parametrize("damage", ["flip", "truncate", "magic", "extend"])
def test_corruption_detected(tmp_path, damage):
    pairs, ref, qer = _batch_with_outputs(200)
    path = str(tmp_path / "c.bswb")
    bsw.write_batch(path, pairs, ref, qer, w=100)
    data = bytearray(open(path, "rb").read())
    if damage == "flip":
        data[128 + 56 * 5 + 3] ^= 0x40
    elif damage == "truncate":
        data = data[:-7]
    elif damage == "magic":
        data[0] ^= 1
    else:
        data += b"\0"
    open(path, "wb").write(bytes(data))
    with pytest.raises(bsw.BswError):
        bsw.read_batch(path)


@pytest.mark.gpu
def test_replay_reproduces_recorded_outputs(tmp_path):
    pairs, ref, qer = _batch_with_outputs(5000, seed=8)
    path = str(tmp_path / "r.bswb")
    bsw.write_batch(path, pairs, ref, qer, w=100)
    h, p2, r2, q2 = bsw.read_batch(path)
    eng = bsw.Engine(h.params)
    got = p2.copy()
    for f in bsw.OUT_FIELDS:
        got[f] = -7
    eng.get_scores(got, r2, q2, h.w, h.cell_bits)
    for f in bsw.OUT_FIELDS:
        assert np.array_equal(got[f], pairs[f]), f
    eng.close()


@pytest.mark.gpu
def test_shim_records_batches(tmp_path):
    """A C++ caller of the upstream-compatible shim with BSW_RECORD set leaves one .bswb per
    getScores call; the recorded outputs equal the oracle's."""
    src = tmp_path / "rec.cpp"
    src.write_text(r'''
#include "bandedSWA_gpu.h"
#include <vector>
int main() {
    int8_t mat[25];
    for (int a = 0; a < 5; ++a) for (int b = 0; b < 5; ++b) mat[a*5+b] = (a == 4 || b == 4) ? -1 : (a == b ? 1 : -4);
    BandedPairWiseSW sw(6, 1, 6, 1, 100, 5, mat, 1, -4, 1);
    const int n = 3000, T = 300, Q = 150;
    std::vector<SeqPair> p(n);
    std::vector<uint8_t> ref(n * T), qer(n * Q);
    uint64_t s = 12345;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 33); };
    for (int i = 0; i < n; ++i) {
        for (int k = 0; k < T; ++k) ref[i*T+k] = rnd() % 4;
        for (int k = 0; k < Q; ++k) qer[i*Q+k] = (rnd() % 10) ? ref[i*T+k] : rnd() % 4;
        memset(&p[i], 0, sizeof(SeqPair));
        p[i].idr = i*T; p[i].idq = i*Q; p[i].len1 = T; p[i].len2 = Q; p[i].h0 = 20 + rnd() % 80; p[i].id = i;
    }
    sw.getScores16(p.data(), ref.data(), qer.data(), n, 1, 100);
    sw.getScores8(p.data(), ref.data(), qer.data(), n, 1, 100);
    return 0;
}
''')
    exe = str(tmp_path / "rec")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"), str(src), "-o", exe,
                    bsw.HIP_LIB, "-Wl,-rpath," + os.path.dirname(bsw.HIP_LIB)], check=True)
    env = dict(os.environ, BSW_RECORD=str(tmp_path / "cap"))
    subprocess.run([exe], check=True, env=env, timeout=300)
    files = sorted(f for f in os.listdir(tmp_path) if f.endswith(".bswb"))
    assert files == ["cap.000000.bswb", "cap.000001.bswb"]
    for f, bits in zip(files, (16, 8)):
        h, pairs, ref, qer = bsw.read_batch(str(tmp_path / f))
        assert h.cell_bits == bits and h.flags == 1 and h.n_pairs == 3000
        want = pairs.copy()
        oracle.get_scores(oracle.make_params(), want, ref, qer, h.w, nthreads=8)
        for fld in bsw.OUT_FIELDS:
            assert np.array_equal(want[fld], pairs[fld]), (f, fld)
