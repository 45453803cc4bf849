"""ctypes binding of the CPU oracle library (oracle/liboracle.so) -- TEST INFRASTRUCTURE.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Exposes the scalar `ksw_extend2` restatement (oracle/ksw_ext_ref.c) and the SSE4.1
inter-pair restatement of upstream's getScores16 (oracle/bsw_sse41.c), both over numpy
arrays in the upstream SeqPair layout.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BSW_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")   # override: `make asan-suite`

SEQPAIR_DTYPE = np.dtype(
    [(n, "<i4") for n in ("idr", "idq", "id", "len1", "len2", "h0", "seqid", "regid",
                          "score", "tle", "gtle", "qle", "gscore", "max_off")]
)
OUT_FIELDS = ("score", "tle", "gtle", "qle", "gscore", "max_off")
assert SEQPAIR_DTYPE.itemsize == 56


class OracleParams(ctypes.Structure):
    _fields_ = [("o_del", ctypes.c_int32), ("e_del", ctypes.c_int32),
                ("o_ins", ctypes.c_int32), ("e_ins", ctypes.c_int32),
                ("zdrop", ctypes.c_int32), ("end_bonus", ctypes.c_int32),
                ("mat", ctypes.c_int8 * 25)]


def make_params(o_del=6, e_del=1, o_ins=6, e_ins=1, zdrop=100, end_bonus=5, mat=None):
    from ksw_ext_ref import bwa_fill_scmat  # noqa: E402  (sibling module)
    p = OracleParams()
    p.o_del, p.e_del, p.o_ins, p.e_ins = o_del, e_del, o_ins, e_ins
    p.zdrop, p.end_bonus = zdrop, end_bonus
    for i, v in enumerate(mat if mat is not None else bwa_fill_scmat()):
        p.mat[i] = v
    return p


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make oracle` (or __graft_entry__.build())")
        _lib = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        _lib.oracle_ksw_extend2.restype = ctypes.c_int
        _lib.oracle_ksw_extend2.argtypes = [ctypes.c_int, P, ctypes.c_int, P, ctypes.c_int, P] + \
            [ctypes.c_int] * 8 + [P] * 5
        _lib.oracle_get_scores.argtypes = [P, P, P, P, ctypes.c_int32, ctypes.c_int32]
        _lib.oracle_get_scores_mt.argtypes = [P, P, P, P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int]
        _lib.sse41_get_scores16.argtypes = [P, P, P, P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int]
        _lib.sse41_get_scores16.restype = ctypes.c_int
        for f in ("avx2_get_scores16", "avx512_get_scores16"):
            getattr(_lib, f).argtypes = [P, P, P, P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int]
            getattr(_lib, f).restype = ctypes.c_int
        _lib.avx2_supported.restype = ctypes.c_int
        _lib.avx512bw_supported.restype = ctypes.c_int
    return _lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def ksw_extend2(query, target, params: OracleParams, w, h0):
    q = np.ascontiguousarray(query, dtype=np.uint8)
    t = np.ascontiguousarray(target, dtype=np.uint8)
    outs = [ctypes.c_int() for _ in range(5)]
    mat = np.frombuffer(bytes(params.mat), dtype=np.int8).copy()
    sc = lib().oracle_ksw_extend2(len(q), _ptr(q), len(t), _ptr(t), 5, _ptr(mat),
                                  params.o_del, params.e_del, params.o_ins, params.e_ins,
                                  w, params.end_bonus, params.zdrop, h0,
                                  *[ctypes.byref(o) for o in outs])
    qle, tle, gtle, gscore, max_off = (o.value for o in outs)
    return sc, qle, tle, gtle, gscore, max_off


def get_scores(params: OracleParams, pairs: np.ndarray, ref: np.ndarray, qer: np.ndarray, w: int,
               nthreads: int = 1):
    """In place on `pairs` (structured SEQPAIR_DTYPE array)."""
    assert pairs.dtype == SEQPAIR_DTYPE and pairs.flags.c_contiguous
    if nthreads > 1:
        lib().oracle_get_scores_mt(ctypes.byref(params), _ptr(pairs), _ptr(ref), _ptr(qer),
                                   len(pairs), w, nthreads)
    else:
        lib().oracle_get_scores(ctypes.byref(params), _ptr(pairs), _ptr(ref), _ptr(qer),
                                len(pairs), w)


def band_cells(params: OracleParams, pairs: np.ndarray, ref: np.ndarray, qer: np.ndarray, w: int) -> int:
    """DP cells the literal ksw_extend2 loop visits on `pairs` (sum of end - beg over rows;
    narrowed band, early z-drop / m == 0 exits) -- one thread, pairs copied."""
    L = lib()
    L.oracle_cells_take.restype = ctypes.c_longlong
    L.oracle_cells_take()
    get_scores(params, pairs.copy(), ref, qer, w)
    return int(L.oracle_cells_take())


def sse41_get_scores16(params: OracleParams, pairs: np.ndarray, ref: np.ndarray, qer: np.ndarray,
                       w: int, nthreads: int = 1) -> int:
    assert pairs.dtype == SEQPAIR_DTYPE and pairs.flags.c_contiguous
    return lib().sse41_get_scores16(ctypes.byref(params), _ptr(pairs), _ptr(ref), _ptr(qer),
                                    len(pairs), w, nthreads)


def simd_get_scores16(isa: str, params: OracleParams, pairs: np.ndarray, ref: np.ndarray, qer: np.ndarray,
                      w: int, nthreads: int = 1) -> int:
    """The same batch restatement at upstream's wider dispatch widths (oracle/bsw_avx512.c): isa
    "avx2" (16 x int16 lanes) or "avx512bw" (32); raises if the host CPU lacks the ISA"""
    assert pairs.dtype == SEQPAIR_DTYPE and pairs.flags.c_contiguous
    L = lib()
    ok = L.avx2_supported() if isa == "avx2" else L.avx512bw_supported() if isa == "avx512bw" else 0
    if not ok:
        raise RuntimeError(f"host CPU lacks {isa}")
    fn = L.avx2_get_scores16 if isa == "avx2" else L.avx512_get_scores16
    return fn(ctypes.byref(params), _ptr(pairs), _ptr(ref), _ptr(qer), len(pairs), w, nthreads)


def simd_supported(isa: str) -> bool:
    L = lib()
    return bool(L.avx2_supported() if isa == "avx2" else L.avx512bw_supported() if isa == "avx512bw" else 0)


def chain2aln(params, opt, ref, reads, read_off, read_len, seeds, seed_read, seed_chain, nthreads=1):
    """oracle_chain2aln (oracle/ext_ref.c): literal per-read mem_chain2aln -> (regions, extended);
    nthreads > 1 splits the reads over pthreads (oracle_chain2aln_mt)."""
    import bsw  # dtypes of the product binding (ALNREG_DTYPE)
    L = lib()
    P = ctypes.c_void_p
    L.oracle_chain2aln.argtypes = [P, P, P, ctypes.c_int64, P, P, P, P, P, P, ctypes.c_int32, P, P]
    L.oracle_chain2aln_mt.argtypes = [P, P, P, ctypes.c_int64, P, P, P, P, P, P, ctypes.c_int32, P, P, ctypes.c_int]
    ptr = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    arrs = [np.ascontiguousarray(x, dtype=d) for x, d in ((ref, np.uint8), (reads, np.uint8), (read_off, np.int64),
                                                           (read_len, np.int32), (seed_read, np.int32),
                                                           (seed_chain, np.int32))]
    seeds = np.ascontiguousarray(seeds)
    out = np.zeros(len(seeds), dtype=bsw.ALNREG_DTYPE)
    ext = np.zeros(len(seeds), dtype=np.int32)
    if nthreads > 1:
        L.oracle_chain2aln_mt(ctypes.byref(params), ctypes.byref(opt), ptr(arrs[0]), len(arrs[0]), ptr(arrs[1]),
                              ptr(arrs[2]), ptr(arrs[3]), ptr(seeds), ptr(arrs[4]), ptr(arrs[5]), len(seeds), ptr(out),
                              ptr(ext), nthreads)
    else:
        L.oracle_chain2aln(ctypes.byref(params), ctypes.byref(opt), ptr(arrs[0]), len(arrs[0]), ptr(arrs[1]),
                           ptr(arrs[2]), ptr(arrs[3]), ptr(seeds), ptr(arrs[4]), ptr(arrs[5]), len(seeds), ptr(out),
                           ptr(ext))
    return out, ext


def extend_seeds(params, opt, ref, reads, read_off, read_len, seeds):
    """oracle/ext_ref.c: per-read CPU restatement of the extension consumer (test checker)."""
    import sys as _sys
    import os as _os
    _sys.path.insert(0, _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                      "bwa-mem2-arm_amd", "py"))
    import bsw as _bsw
    L = lib()
    P = ctypes.c_void_p
    L.oracle_extend_seeds.argtypes = [P, P, P, ctypes.c_int64, P, P, P, P, ctypes.c_int32, P]
    ref = np.ascontiguousarray(ref, dtype=np.uint8)
    reads = np.ascontiguousarray(reads, dtype=np.uint8)
    read_off = np.ascontiguousarray(read_off, dtype=np.int64)
    read_len = np.ascontiguousarray(read_len, dtype=np.int32)
    seeds = np.ascontiguousarray(seeds, dtype=_bsw.SEED_DTYPE)
    out = np.zeros(len(seeds), dtype=_bsw.ALNREG_DTYPE)
    ptr = lambda a: ctypes.c_void_p(a.ctypes.data)
    L.oracle_extend_seeds(ctypes.byref(params), ctypes.byref(opt), ptr(ref), len(ref), ptr(reads),
                          ptr(read_off), ptr(read_len), ptr(seeds), len(seeds), ptr(out))
    return out


KSWR_DTYPE = np.dtype([(n, "<i4") for n in ("score", "te", "qe", "score2", "te2", "tb", "qb")])


class _Kswr(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in KSWR_DTYPE.names]


def ksw_align2(query, target, mat, o_del, e_del, o_ins, e_ins, xtra):
    """oracle/ksw_align_ref.c: literal striped ksw_align2 (one pair) -> list of 7 ints."""
    L = lib()
    P = ctypes.c_void_p
    L.oracle_ksw_align2.restype = _Kswr
    L.oracle_ksw_align2.argtypes = [ctypes.c_int, P, ctypes.c_int, P, ctypes.c_int, P] + [ctypes.c_int] * 5
    q = np.ascontiguousarray(query, dtype=np.uint8)
    t = np.ascontiguousarray(target, dtype=np.uint8)
    m = np.ascontiguousarray(mat, dtype=np.int8)
    r = L.oracle_ksw_align2(len(q), _ptr(q), len(t), _ptr(t), 5, _ptr(m), o_del, e_del, o_ins, e_ins, xtra)
    return [getattr(r, n) for n in KSWR_DTYPE.names]


def ksw_align2_batch(pairs, ref, qer, mat, o_del=6, e_del=1, o_ins=6, e_ins=1, nthreads=1):
    """Batch over SeqPairs (len1 = target, len2 = query, h0 = xtra) -> KSWR_DTYPE array."""
    assert pairs.dtype == SEQPAIR_DTYPE and pairs.flags.c_contiguous
    L = lib()
    P = ctypes.c_void_p
    L.oracle_ksw_align2_batch.argtypes = [P, P, P, ctypes.c_int, P] + [ctypes.c_int] * 4 + [P, ctypes.c_int]
    m = np.ascontiguousarray(mat, dtype=np.int8)
    out = np.zeros(len(pairs), dtype=KSWR_DTYPE)
    L.oracle_ksw_align2_batch(_ptr(pairs), _ptr(ref), _ptr(qer), len(pairs), _ptr(m), o_del, e_del, o_ins,
                              e_ins, _ptr(out), nthreads)
    return out


def ksw_global2(query, target, mat, o_del, e_del, o_ins, e_ins, w):
    """oracle/ksw_global_ref.c: literal ksw_global2 (one pair) -> (score, [(op, len), ...])."""
    L = lib()
    P = ctypes.c_void_p
    L.oracle_ksw_global2.restype = ctypes.c_int
    L.oracle_ksw_global2.argtypes = [ctypes.c_int, P, ctypes.c_int, P, ctypes.c_int, P] + \
        [ctypes.c_int] * 5 + [P, P]
    q = np.ascontiguousarray(query, dtype=np.uint8)
    t = np.ascontiguousarray(target, dtype=np.uint8)
    m = np.ascontiguousarray(mat, dtype=np.int8)
    nc = ctypes.c_int(0)
    cg = ctypes.POINTER(ctypes.c_uint32)()
    sc = L.oracle_ksw_global2(len(q), _ptr(q), len(t), _ptr(t), 5, _ptr(m), o_del, e_del, o_ins, e_ins,
                              w, ctypes.byref(nc), ctypes.byref(cg))
    ops = [(cg[k] & 0xf, cg[k] >> 4) for k in range(nc.value)]
    if cg:
        ctypes.CDLL(None).free(cg)
    return sc, ops


def ksw_global2_batch(pairs, ref, qer, mat, o_del=6, e_del=1, o_ins=6, e_ins=1, stride=64, nthreads=1):
    """Batch over SeqPairs (len1 = target, len2 = query, h0 = w) -> (score, cigar[n, stride],
    n_cigar) with n_cigar -1 (more than `stride` ops) / -2 (qlen < tlen - w, undefined);
    stride 0: scores only (cigar None, n_cigar zeros)."""
    assert pairs.dtype == SEQPAIR_DTYPE and pairs.flags.c_contiguous
    L = lib()
    P = ctypes.c_void_p
    L.oracle_ksw_global2_batch.argtypes = [P, P, P, ctypes.c_int, P] + [ctypes.c_int] * 4 + \
        [P, P, ctypes.c_int, P, ctypes.c_int]
    m = np.ascontiguousarray(mat, dtype=np.int8)
    n = len(pairs)
    score = np.zeros(n, dtype=np.int32)
    ncig = np.zeros(n, dtype=np.int32)
    cig = np.zeros((n, stride), dtype=np.uint32) if stride > 0 else None
    L.oracle_ksw_global2_batch(_ptr(pairs), _ptr(ref), _ptr(qer), n, _ptr(m), o_del, e_del, o_ins, e_ins,
                               _ptr(score), _ptr(cig) if cig is not None else None, stride, _ptr(ncig),
                               nthreads)
    return score, cig, ncig


# ---- FM-index SMEM seeding (oracle/fmi_ref.c: bwt_smem1a / bwt_seed_strategy1 / mem_collect_intv)

BWTINTV_DTYPE = np.dtype([("k", "<u8"), ("l", "<u8"), ("s", "<u8"), ("info", "<u8")])   # bwa's bwtintv_t


class _MemOpt(ctypes.Structure):
    _fields_ = [("min_seed_len", ctypes.c_int32), ("split_width", ctypes.c_int32),
                ("max_mem_intv", ctypes.c_int32), ("split_factor", ctypes.c_float)]


def mem_opt(min_seed_len=19, split_width=10, max_mem_intv=20, split_factor=1.5):
    """bwa mem defaults: -k 19, split_width 10, max_mem_intv 20, -r 1.5"""
    return _MemOpt(min_seed_len, split_width, max_mem_intv, split_factor)


class FmiRef:
    """The oracle's FM-index of ref + reverse-complement(ref) (comparison-sorted suffix array,
    prefix-count occurrence table) and its SMEM passes."""

    def __init__(self, ref, sa=None, lean=False, nthreads=1):
        """sa: build from this suffix array of T$ instead of sorting (bench CPU leg only).
        lean: the genome-scale form (oracle_fmi_build_lean, needs sa): occurrence checkpoints
        every 64 rows and an SA sampled every 32 rows resolved by LF walks, ~1.8 B per row."""
        L = lib()
        P = ctypes.c_void_p
        L.oracle_fmi_sizeof.restype = ctypes.c_size_t
        L.oracle_fmi_build.argtypes = [P, ctypes.c_int64, P]
        L.oracle_fmi_build.restype = ctypes.c_int
        for f in ("oracle_fmi_n", "oracle_fmi_sentinel"):
            getattr(L, f).restype = ctypes.c_int64
            getattr(L, f).argtypes = [P]
        L.oracle_fmi_count.argtypes = [P, P]
        L.oracle_fmi_sa.argtypes = [P, P]
        L.oracle_fmi_bwt.argtypes = [P, P]
        L.oracle_fmi_free.argtypes = [P]
        L.oracle_collect_intv_mt.argtypes = [P, P, P, P, P, ctypes.c_int32, P, ctypes.c_int32, P, ctypes.c_int]
        self._buf = ctypes.create_string_buffer(L.oracle_fmi_sizeof())
        self.ref = np.ascontiguousarray(ref, dtype=np.uint8)
        self.lean = bool(lean)
        if lean:
            L.oracle_fmi_build_lean.argtypes = [P, ctypes.c_int64, P, ctypes.c_int, P]
            sa = np.ascontiguousarray(sa, dtype=np.int64)
            assert len(sa) == 2 * len(self.ref) + 1
            rc = L.oracle_fmi_build_lean(_ptr(self.ref), len(self.ref), _ptr(sa), int(nthreads), self._buf)
        elif sa is not None:
            L.oracle_fmi_build_with_sa.argtypes = [P, ctypes.c_int64, P, P]
            sa = np.ascontiguousarray(sa, dtype=np.int64)
            assert len(sa) == 2 * len(self.ref) + 1
            rc = L.oracle_fmi_build_with_sa(_ptr(self.ref), len(self.ref), _ptr(sa), self._buf)
        else:
            rc = L.oracle_fmi_build(_ptr(self.ref), len(self.ref), self._buf)
        if rc != 0:
            raise ValueError("oracle_fmi_build failed (codes must be 0..3)")
        self.n = L.oracle_fmi_n(self._buf)
        self.sentinel = L.oracle_fmi_sentinel(self._buf)
        self.count = np.zeros(5, dtype=np.int64)
        L.oracle_fmi_count(self._buf, _ptr(self.count))

    def sa_rows(self, rows):
        """SA at the given rows (bwt_sa: LF walks in the lean form)"""
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        out = np.zeros(len(rows), dtype=np.int64)
        lib().oracle_fmi_sa_rows.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        lib().oracle_fmi_sa_rows(self._buf, _ptr(rows), len(rows), _ptr(out))
        return out

    def sa(self):
        a = np.zeros(self.n + 1, dtype=np.int64)
        lib().oracle_fmi_sa(self._buf, _ptr(a))
        return a

    def bwt(self):
        a = np.zeros(self.n + 1, dtype=np.uint8)
        lib().oracle_fmi_bwt(self._buf, _ptr(a))
        return a

    def collect_intv(self, reads, off, lens, cap=256, opt=None, nthreads=1):
        """mem_collect_intv per read -> (intervals [n, cap] BWTINTV_DTYPE, counts [n])"""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        n = len(lens)
        out = np.zeros((n, cap), dtype=BWTINTV_DTYPE)
        cnt = np.zeros(n, dtype=np.int32)
        o = opt if opt is not None else mem_opt()
        lib().oracle_collect_intv_mt(self._buf, ctypes.byref(o), _ptr(reads), _ptr(off), _ptr(lens), n,
                                     _ptr(out), cap, _ptr(cnt), nthreads)
        return out, cnt

    @staticmethod
    def counters(reset=False):
        """(backward extensions, 64-row blocks they touched) since the last reset"""
        c = np.zeros(2, dtype=np.uint64)
        lib().oracle_fmi_counters.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib().oracle_fmi_counters(_ptr(c), int(reset))
        return int(c[0]), int(c[1])

    def __del__(self):
        try:
            lib().oracle_fmi_free(self._buf)
        except Exception:
            pass


# ---- seeds -> chains (oracle/chain_ref.c: mem_chain + mem_chain_flt)

class ChainOpt(ctypes.Structure):
    """bsw_chain_opt_t (include/bsw_fmi.h)"""
    _fields_ = [("max_occ", ctypes.c_int32), ("w", ctypes.c_int32), ("max_chain_gap", ctypes.c_int32),
                ("min_chain_weight", ctypes.c_int32), ("min_seed_len", ctypes.c_int32),
                ("max_chain_extend", ctypes.c_int32), ("drop_ratio", ctypes.c_float), ("mask_level", ctypes.c_float)]


def chain_opt(**kw):
    """bwa mem defaults: -c 500 -w 100, max_chain_gap 10000, -W 0, -k 19, max_chain_extend 1 << 30,
    -D 0.5, mask_level 0.5"""
    o = ChainOpt(500, 100, 10000, 0, 19, 1 << 30, 0.5, 0.5)
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def mem_chain(sa, l_pac, read_len, mems, n_mems, opt=None):
    """oracle_mem_chain over every read: (seeds SEED layout, seed_read, seed_chain) as bsw_fmi.h.
    sa: the suffix array of T$ (numpy), or an FmiRef whose bwt_sa resolves the rows (lean form)."""
    import bsw as _bsw
    L = lib()
    P = ctypes.c_void_p
    fn = L.oracle_mem_chain_fmi if isinstance(sa, FmiRef) else L.oracle_mem_chain
    fn.restype = ctypes.c_int64
    fn.argtypes = [P, P, ctypes.c_int64, P, ctypes.c_int32, P, ctypes.c_int32, P, P, P, P, ctypes.c_int64]
    o = opt if opt is not None else chain_opt()
    src = sa._buf if isinstance(sa, FmiRef) else None
    if src is None:
        sa = np.ascontiguousarray(sa, dtype=np.int64)
    read_len = np.ascontiguousarray(read_len, dtype=np.int32)
    mems = np.ascontiguousarray(mems)
    n_mems = np.ascontiguousarray(n_mems, dtype=np.int32)
    n, cap = mems.shape
    cnt = 0
    for _ in range(2):
        seeds = np.zeros(max(cnt, 1), dtype=_bsw.SEED_DTYPE)
        sr = np.zeros(max(cnt, 1), dtype=np.int32)
        sc = np.zeros(max(cnt, 1), dtype=np.int32)
        need = fn(ctypes.byref(o), src if src is not None else _ptr(sa), l_pac, _ptr(read_len), n, _ptr(mems), cap,
                  _ptr(n_mems), _ptr(seeds), _ptr(sr), _ptr(sc), cnt)
        if need <= cnt:
            return seeds[:need], sr[:need], sc[:need]
        cnt = need
    raise RuntimeError("oracle_mem_chain: seed count changed between passes")
