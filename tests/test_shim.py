"""The upstream-compatible C++ shim (include/bandedSWA_gpu.h) called from compiled C++: the
scalar members `scalarBandedSWAWrapper` (batch) and `scalarBandedSWA` (one pair, the
ksw_extend2-shaped signature) return the oracle's outputs, and the shim's error convention
(stderr + exit(EXIT_FAILURE)) fires on a bad batch.  The getScores16/8 members are covered by
tests/test_batch_file.py::test_shim_records_batches."""

import os
import subprocess

import numpy as np
import pytest

import bsw
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

PROG = r'''
#include "bandedSWA_gpu.h"
#include <cstdio>
#include <string>
#include <vector>
static void dump(const char *path, const void *p, size_t n) {
    FILE *f = fopen(path, "wb"); fwrite(p, 1, n, f); fclose(f);
}
int main(int argc, char **argv) {
    const char *dir = argv[1];
    const int bad = argc > 2;
    int8_t mat[25];
    for (int a = 0; a < 5; ++a) for (int b = 0; b < 5; ++b) mat[a*5+b] = (a == 4 || b == 4) ? -1 : (a == b ? 1 : -4);
    BandedPairWiseSW sw(6, 1, 6, 1, 100, 5, mat, 1, -4, 4);
    const int n = 2000;
    std::vector<SeqPair> p(n);
    std::vector<uint8_t> ref, qer;
    uint64_t s = 777;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 33); };
    for (int i = 0; i < n; ++i) {
        const int T = rnd() % 320, Q = rnd() % 200;            // lengths 0.. (incl. > 160: wide kernel)
        memset(&p[i], 0, sizeof(SeqPair));
        p[i].idr = (int)ref.size(); p[i].idq = (int)qer.size();
        p[i].len1 = T; p[i].len2 = Q; p[i].h0 = rnd() % 120; p[i].id = i;
        for (int k = 0; k < T; ++k) ref.push_back(rnd() % 50 ? rnd() % 4 : 4);
        for (int k = 0; k < Q; ++k) qer.push_back((k < T && rnd() % 8) ? ref[p[i].idr + k] : rnd() % 5);
    }
    if (bad) p[7].len1 = 40000;                                 // > BSW_MAX_LEN: engine error
    std::vector<SeqPair> a = p, b = p;
    sw.scalarBandedSWAWrapper(a.data(), ref.data(), qer.data(), n, 4, 100);
    for (int i = 0; i < n; ++i) {                              // one pair per call, upstream's
        int qle, tle, gtle, gscore, moff;                      // ksw_extend2-shaped member
        b[i].score = sw.scalarBandedSWA(b[i].len2, qer.data() + b[i].idq, b[i].len1, ref.data() + b[i].idr,
                                        37, b[i].h0, &qle, &tle, &gtle, &gscore, &moff);
        b[i].qle = qle; b[i].tle = tle; b[i].gtle = gtle; b[i].gscore = gscore; b[i].max_off = moff;
    }
    std::string d(dir);
    dump((d + "/pairs.bin").c_str(), p.data(), n * sizeof(SeqPair));
    dump((d + "/wrapper.bin").c_str(), a.data(), n * sizeof(SeqPair));
    dump((d + "/single.bin").c_str(), b.data(), n * sizeof(SeqPair));
    dump((d + "/ref.bin").c_str(), ref.data(), ref.size());
    dump((d + "/qer.bin").c_str(), qer.data(), qer.size());
    return 0;
}
'''


def _build(tmp_path):
    src = tmp_path / "scalar.cpp"
    src.write_text(PROG)
    exe = str(tmp_path / "scalar")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"), str(src), "-o", exe,
                    bsw.HIP_LIB, "-Wl,-rpath," + os.path.dirname(bsw.HIP_LIB)], check=True)
    return exe


def test_shim_scalar_members(tmp_path):
    exe = _build(tmp_path)
    subprocess.run([exe, str(tmp_path)], check=True, timeout=300)
    load = lambda nm, dt: np.fromfile(str(tmp_path / nm), dtype=dt)  # noqa: E731
    pairs = load("pairs.bin", bsw.SEQPAIR_DTYPE)
    ref, qer = load("ref.bin", np.uint8), load("qer.bin", np.uint8)
    for name, w in (("wrapper.bin", 100), ("single.bin", 37)):
        got = load(name, bsw.SEQPAIR_DTYPE)
        want = pairs.copy()
        oracle.get_scores(oracle.make_params(), want, ref, qer, w, nthreads=8)
        for f in bsw.OUT_FIELDS:
            assert np.array_equal(want[f], got[f]), (name, f, int((want[f] != got[f]).sum()))
    assert (pairs["len2"] > 160).any()                          # the wide kernel took part


def test_shim_error_convention(tmp_path):
    """A pair over BSW_MAX_LEN: the shim prints the engine error and exits with EXIT_FAILURE,
    as upstream's BandedPairWiseSW does on internal failure."""
    exe = _build(tmp_path)
    r = subprocess.run([exe, str(tmp_path), "bad"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 1
    assert "scalarBandedSWAWrapper failed" in r.stderr and "(-34)" in r.stderr


PROG_MT = r'''
#include "bandedSWA_gpu.h"
#include <cstdio>
#include <string>
#include <thread>
#include <vector>
// kt_for-style callers: 8 worker threads, each hands getScores16 / getScores8 many small
// batches (1000 pairs, upstream's per-task sizes), then one large batch of all pairs
int main(int argc, char **argv) {
    const char *dir = argv[1];
    int8_t mat[25];
    for (int a = 0; a < 5; ++a) for (int b = 0; b < 5; ++b) mat[a*5+b] = (a == 4 || b == 4) ? -1 : (a == b ? 1 : -4);
    BandedPairWiseSW sw(6, 1, 6, 1, 100, 5, mat, 1, -4, 8);
    const int n = 200000, task = 1000, nt = 8;
    std::vector<SeqPair> p(n);
    std::vector<uint8_t> ref, qer;
    uint64_t s = 4242;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 33); };
    for (int i = 0; i < n; ++i) {
        const int T = 200 + rnd() % 120, Q = 100 + rnd() % 60;
        memset(&p[i], 0, sizeof(SeqPair));
        p[i].idr = (int)ref.size(); p[i].idq = (int)qer.size();
        p[i].len1 = T; p[i].len2 = Q; p[i].h0 = 19 + rnd() % 80; p[i].id = i;
        for (int k = 0; k < T; ++k) ref.push_back(rnd() % 100 ? rnd() % 4 : 4);
        for (int k = 0; k < Q; ++k) qer.push_back(rnd() % 16 ? ref[p[i].idr + k] : rnd() % 4);
    }
    std::vector<SeqPair> small = p, big = p;
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int a = t * task; a < n; a += nt * task) {
                const int m = std::min(task, n - a);
                if ((a / task) & 1) sw.getScores8(small.data() + a, ref.data(), qer.data(), m, 1, 100);
                else sw.getScores16(small.data() + a, ref.data(), qer.data(), m, 1, 100);
            }
        });
    for (auto &x : th) x.join();
    sw.getScores16(big.data(), ref.data(), qer.data(), n, nt, 100);
    std::string d(dir);
    auto dump = [&](const char *nm, const void *q, size_t b) {
        FILE *f = fopen((d + nm).c_str(), "wb"); fwrite(q, 1, b, f); fclose(f);
    };
    dump("/pairs.bin", p.data(), n * sizeof(SeqPair));
    dump("/small.bin", small.data(), n * sizeof(SeqPair));
    dump("/big.bin", big.data(), n * sizeof(SeqPair));
    dump("/ref.bin", ref.data(), ref.size());
    dump("/qer.bin", qer.data(), qer.size());
    return 0;
}
'''


@pytest.mark.parametrize("gmap", ["0,0", "0,0,0,0"])
def test_shim_multi_gpu_rehearsal(tmp_path, gmap):
    """The shim's multi-GPU path (BSW_GPUS / BSW_GPU_MAP -> bsw_create_on) with 2 and 4 logical
    devices on the box's one GPU: 8 kt_for-style threads of 1000-pair getScores16/8 calls (each
    runs whole on the least-busy device) and one 200K-pair call (split over every device) both
    equal the oracle."""
    src = tmp_path / "mt.cpp"
    src.write_text(PROG_MT)
    exe = str(tmp_path / "mt")
    subprocess.run(["g++", "-O1", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    exe, bsw.HIP_LIB, "-Wl,-rpath," + os.path.dirname(bsw.HIP_LIB)], check=True)
    env = dict(os.environ, BSW_GPUS=str(len(gmap.split(","))), BSW_GPU_MAP=gmap)
    subprocess.run([exe, str(tmp_path)], check=True, timeout=300, env=env)
    load = lambda nm, dt: np.fromfile(str(tmp_path / nm), dtype=dt)  # noqa: E731
    pairs = load("pairs.bin", bsw.SEQPAIR_DTYPE)
    ref, qer = load("ref.bin", np.uint8), load("qer.bin", np.uint8)
    want = pairs.copy()
    oracle.get_scores(oracle.make_params(), want, ref, qer, 100, nthreads=16)
    for name in ("small.bin", "big.bin"):
        got = load(name, bsw.SEQPAIR_DTYPE)
        for f in bsw.OUT_FIELDS:
            assert np.array_equal(want[f], got[f]), (gmap, name, f, int((want[f] != got[f]).sum()))
