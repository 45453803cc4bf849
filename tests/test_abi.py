"""C-ABI checks that need no GPU: the product library loads, exports every symbol the
public headers declare, SeqPair is byte-compatible with upstream's 56-byte layout, and the
argument validation / error strings behave (no compute call is made here)."""

import ctypes
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

import bsw
from conftest import ROOT

HEADERS = [os.path.join(ROOT, "include", h) for h in ("bsw.h", "bsw_ext.h", "bsw_batch.h", "bsw_mate.h", "bsw_global.h", "bsw_fmi.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(bswb?_[a-z_0-9]+)\s*\(", src))
        names -= set(re.findall(r"static inline \w+ (bswb?_[a-z_0-9]+)\s*\(", src))   # header-only helpers
    return sorted(names)


def test_header_declares_expected_api():
    assert set(declared_functions()) == set(bsw.ABI_SYMBOLS)


def test_library_exports_all_declared_symbols():
    lib = bsw.hip_lib()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", bsw.HIP_LIB], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (bswb?_\w+)", out))
    assert set(declared_functions()) <= exported


def test_library_links_hip_runtime_not_torch():
    out = subprocess.run(["readelf", "-d", bsw.HIP_LIB], capture_output=True, text=True).stdout
    assert "libamdhip64.so" in out
    assert "torch" not in out and "python" not in out


def test_kernels_are_gfx950_code_objects(tmp_path):
    # on a copy: --offloading extracts the code objects next to the file it reads
    lib = tmp_path / "lib.so"
    shutil.copyfile(bsw.HIP_LIB, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    text = out.stdout + out.stderr
    assert "gfx950" in text


def test_seqpair_layout():
    assert bsw.SEQPAIR_DTYPE.itemsize == 56
    names = bsw.SEQPAIR_DTYPE.names
    assert names[:6] == ("idr", "idq", "id", "len1", "len2", "h0")
    assert names[8:] == bsw.OUT_FIELDS
    assert bsw.SEQPAIR_DTYPE.fields["score"][1] == 32 and bsw.SEQPAIR_DTYPE.fields["max_off"][1] == 52
    hdr = open(os.path.join(ROOT, "include", "bsw_seqpair.h")).read()
    assert "sizeof(SeqPair) == 56" in hdr


def test_params_default_and_abi_version():
    lib = bsw.hip_lib()
    p = bsw.Params()
    lib.bsw_params_default(ctypes.byref(p))
    assert (p.o_del, p.e_del, p.o_ins, p.e_ins, p.zdrop, p.end_bonus) == (6, 1, 6, 1, 100, 5)
    mat = np.frombuffer(bytes(p.mat), np.int8).reshape(5, 5)
    assert mat[0, 0] == 1 and mat[0, 1] == -4 and mat[4, 4] == -1 and mat[2, 4] == -1
    assert lib.bsw_abi_version() == 8
    ref = bsw.default_params()
    assert bytes(ref.mat) == bytes(p.mat)


def test_strerror_and_invalid_arguments():
    lib = bsw.hip_lib()
    for code in (0, -22, -12, -19, -5, -34):
        assert lib.bsw_strerror(code)
    # invalid arguments are rejected before any device work
    P = ctypes.c_void_p
    assert lib.bsw_create(None, 0, 1, ctypes.byref(P())) == -22
    bad = bsw.default_params()
    bad.e_del = 0
    assert lib.bsw_create(ctypes.byref(bad), 0, 1, ctypes.byref(P())) == -22
    assert lib.bsw_create(ctypes.byref(bsw.default_params()), 0, 0, ctypes.byref(P())) == -22
    assert lib.bsw_get_scores(None, None, None, None, 0, 100, 16) == -22
    st = bsw.Stats()
    assert lib.bsw_last_stats(None, ctypes.byref(st)) == -22


def test_create_without_gpu_fails_cleanly():
    """Here (no GPU) bsw_create must return BSW_E_NODEV, never crash or fall back."""
    import hiprt
    if hiprt.device_count() > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    lib = bsw.hip_lib()
    ctx = ctypes.c_void_p()
    rc = lib.bsw_create(ctypes.byref(bsw.default_params()), 0, 1, ctypes.byref(ctx))
    assert rc == -19 and not ctx.value
    with pytest.raises(bsw.BswError):
        bsw.Engine()


def test_shim_header_compiles_against_c_abi(tmp_path):
    """The upstream-compatible C++ shim (include/bandedSWA_gpu.h) compiles and links."""
    src = tmp_path / "shim.cpp"
    src.write_text('#include "bandedSWA_gpu.h"\nint main(){ int8_t mat[25]; for(int i=0;i<25;++i) mat[i]=-1;\n'
                   ' BandedPairWiseSW* p = nullptr; (void)p; (void)mat; return 0; }\n')
    r = subprocess.run(["g++", "-std=c++14", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                        str(tmp_path / "shim"), bsw.HIP_LIB, "-Wl,-rpath," + os.path.dirname(bsw.HIP_LIB)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_ext_header_layouts_compile(tmp_path):
    """include/bsw_ext.h structs match the Python mirrors (compiled by gcc, no GPU)."""
    src = tmp_path / "t.c"
    src.write_text(
        '#include <stddef.h>\n#include "bsw_ext.h"\n'
        "_Static_assert(sizeof(bsw_seed_t) == 16, \"seed\");\n"
        "_Static_assert(sizeof(bsw_alnreg_t) == 40, \"alnreg\");\n"
        "_Static_assert(offsetof(bsw_alnreg_t, qb) == 16, \"qb\");\n"
        "_Static_assert(offsetof(bsw_alnreg_t, seedlen0) == 36, \"seedlen0\");\n"
        "_Static_assert(sizeof(bsw_ext_opt_t) == 24, \"opt\");\n")
    r = subprocess.run(["gcc", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert bsw.SEED_DTYPE.itemsize == 16 and bsw.ALNREG_DTYPE.itemsize == 40
    assert ctypes.sizeof(bsw.ExtOpt) == 24


def _static_cells(q, t, w):
    return sum(max(0, min(q, i + w + 1) - max(0, i - w)) for i in range(t))


def test_split_by_cells_balances_static_band_cells():
    """bsw_split_by_cells (host-only): contiguous parts of ~equal static band cells; the split
    the n_gpus engine and bench.py's strong-scaling ranks use."""
    rng = np.random.default_rng(5)
    n, w = 3000, 40
    pairs = np.zeros(n, dtype=bsw.SEQPAIR_DTYPE)
    pairs["len2"] = rng.integers(0, 200, n)
    pairs["len1"] = rng.integers(0, 400, n)
    pairs["len2"][:1000] = 20                     # a cheap head: a count split would be unbalanced
    cost = np.array([64 + _static_cells(int(q), int(t), w) for q, t in zip(pairs["len2"], pairs["len1"])])
    for parts in (1, 2, 3, 8):
        cut = bsw.split_by_cells(pairs, w, parts)
        assert cut[0] == 0 and cut[-1] == n and np.all(np.diff(cut) >= 0)
        shares = [cost[cut[k]:cut[k + 1]].sum() for k in range(parts)]
        assert max(shares) - min(shares) <= 2 * cost.max(), (parts, shares)
    # closed form == the row sum on the C2 shape (25,100 cells: SURVEY.md §8(d))
    one = np.zeros(2, dtype=bsw.SEQPAIR_DTYPE)
    one["len2"], one["len1"] = 150, 300
    assert _static_cells(150, 300, 100) == 25_100
    assert list(bsw.split_by_cells(one, 100, 2)) == [0, 1, 2]
    with pytest.raises(bsw.BswError):
        bsw.split_by_cells(one, 100, 0)
