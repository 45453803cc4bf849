"""ctypes binding of the product C ABI (include/bsw.h -> lib/libbsw_hip.so) and of the
synthetic-batch tool (lib/libbsw_synth.so).

This is plumbing for tests and bench.py: the product is the C ABI / C++ shim; PyTorch
is used only for device memory, streams and torch.distributed.  Loading fails loudly
when the HIP library is missing -- there is no CPU fallback anywhere in this module.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(PKG, "lib")
HIP_LIB = os.environ.get("BSW_HIP_LIB") or os.path.join(LIBDIR, "libbsw_hip.so")   # override: experiment builds
SYNTH_LIB = os.environ.get("BSW_SYNTH_LIB") or os.path.join(LIBDIR, "libbsw_synth.so")   # override: `make asan-suite`

SEQPAIR_DTYPE = np.dtype(
    [(n, "<i4") for n in ("idr", "idq", "id", "len1", "len2", "h0", "seqid", "regid",
                          "score", "tle", "gtle", "qle", "gscore", "max_off")]
)
OUT_FIELDS = ("score", "tle", "gtle", "qle", "gscore", "max_off")
assert SEQPAIR_DTYPE.itemsize == 56

# Every symbol include/bsw.h declares (tests check the library exports all of them).
ABI_SYMBOLS = ("bsw_params_default", "bsw_create", "bsw_create_on", "bsw_destroy", "bsw_get_scores",
               "bsw_get_scores_device", "bsw_last_stats", "bsw_strerror", "bsw_abi_version",
               "bsw_pack_batch", "bsw_get_scores_packed_device",
               "bsw_ext_opt_default", "bsw_extend_seeds", "bsw_ext_last_stats",
               "bswb_write", "bswb_read_header", "bswb_read",
               "bsw_ksw_align2", "bsw_ksw_align2_device", "bsw_mate_last_stats",
               "bsw_ksw_global2", "bsw_ksw_global2_device", "bsw_global_last_stats",
               "bsw_set_reference", "bsw_extend_seeds_device", "bsw_set_option",
               "bsw_split_by_cells", "bsw_chain2aln", "bsw_chain2aln_device", "bsw_chain_last_stats",
               "bsw_chain2aln_resident", "bsw_mem_opt_default", "bsw_fmi_build", "bsw_fmi_destroy", "bsw_fmi_get_info", "bsw_fmi_copy_sa",
               "bsw_fmi_copy_bwt", "bsw_mem_collect_intv", "bsw_mem_collect_intv_device", "bsw_fmi_sa_device",
               "bsw_fmi_last_kernel_ms", "bsw_chain_opt_default", "bsw_mem_chain_device", "bsw_fmi_build2", "bsw_fmi_check")

# include/bsw.h engine options (bsw_set_option)
OPT_KERNEL8, OPT_FORK, OPT_SORTKEY, OPT_GLOB_BAND, OPT_EXT_CHUNK, OPT_HOST_CHUNK, OPT_LONG, OPT_HOST_PACK = 1, 2, 3, 4, 5, 6, 7, 8
OPT_SMALL_BATCH = 9
OPT_SPLIT_MIN = 10
OPT_COALESCE = 11
OPT_COALESCE_LEADERS = 12
OPT_GROUP_KERNEL = 13
OPT_MID_BATCH = 14
OPT_COALESCE_LINGER = 16
OPT_GQ32_MAX = 18
OPT_TEST_MISROUTE = 100
OPT_TEST_FAIL_ALLOC = 101

# include/bsw_ext.h structs
SEED_DTYPE = np.dtype([("rbeg", np.int64), ("qbeg", np.int32), ("len", np.int32)])
ALNREG_DTYPE = np.dtype([("rb", np.int64), ("re", np.int64), ("qb", np.int32), ("qe", np.int32),
                         ("score", np.int32), ("truesc", np.int32), ("w", np.int32),
                         ("seedlen0", np.int32)])
assert SEED_DTYPE.itemsize == 16 and ALNREG_DTYPE.itemsize == 40

# include/bsw_mate.h
KSW_XBYTE, KSW_XSTOP, KSW_XSUBO, KSW_XSTART = 0x10000, 0x20000, 0x40000, 0x80000
KSWR_DTYPE = np.dtype([(n, "<i4") for n in ("score", "te", "qe", "score2", "te2", "tb", "qb")])
assert KSWR_DTYPE.itemsize == 28


class Params(ctypes.Structure):
    """Mirror of bsw_params_t (include/bsw.h)."""
    _fields_ = [("o_del", ctypes.c_int32), ("e_del", ctypes.c_int32),
                ("o_ins", ctypes.c_int32), ("e_ins", ctypes.c_int32),
                ("zdrop", ctypes.c_int32), ("end_bonus", ctypes.c_int32),
                ("mat", ctypes.c_int8 * 25), ("w_match", ctypes.c_int8),
                ("w_mismatch", ctypes.c_int8), ("w_ambig", ctypes.c_int8)]


class Stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_float), ("n_i16", ctypes.c_int32),
                ("n_u8", ctypes.c_int32), ("n_wide", ctypes.c_int32),
                ("n_launches", ctypes.c_int32), ("n_packed", ctypes.c_int32),
                ("stage_ms", ctypes.c_float), ("host_ms", ctypes.c_float), ("n_wave", ctypes.c_int32),
                ("n_devices", ctypes.c_int32), ("n_group", ctypes.c_int32),
                ("recovery", ctypes.c_int32)]


def default_params(a=1, b=4, o_del=6, e_del=1, o_ins=6, e_ins=1, zdrop=100, end_bonus=5,
                   ambig=-1, mat=None) -> Params:
    p = Params()
    p.o_del, p.e_del, p.o_ins, p.e_ins = o_del, e_del, o_ins, e_ins
    p.zdrop, p.end_bonus = zdrop, end_bonus
    if mat is None:
        mat = [ambig if (t == 4 or q == 4) else (a if t == q else -b)
               for t in range(5) for q in range(5)]
    for i, v in enumerate(mat):
        p.mat[i] = int(v)
    p.w_match, p.w_mismatch, p.w_ambig = a, -b, ambig
    return p


class BswError(RuntimeError):
    pass


_hip = None


def hip_lib():
    """Load libbsw_hip.so (raises if it was not built: no silent fallback)."""
    global _hip
    if _hip is None:
        if not os.path.exists(HIP_LIB):
            raise BswError(f"{HIP_LIB} not built: run `make` or __graft_entry__.build()")
        L = ctypes.CDLL(HIP_LIB)
        P = ctypes.c_void_p
        L.bsw_params_default.argtypes = [P]
        L.bsw_create.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(P)]
        L.bsw_create_on.argtypes = [P, P, ctypes.c_int, ctypes.POINTER(P)]
        L.bsw_destroy.argtypes = [P]
        L.bsw_get_scores.argtypes = [P, P, P, P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int]
        L.bsw_get_scores_device.argtypes = [P, P, P, P, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int, P]
        L.bsw_last_stats.argtypes = [P, P]
        L.bsw_strerror.restype = ctypes.c_char_p
        L.bsw_strerror.argtypes = [ctypes.c_int]
        L.bswb_write.argtypes = [ctypes.c_char_p, P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int, P,
                                 ctypes.c_int64, P, ctypes.c_int64, P, ctypes.c_int64]
        L.bswb_read_header.argtypes = [ctypes.c_char_p, P]
        L.bswb_read.argtypes = [ctypes.c_char_p, P, P, P, P]
        L.bsw_ext_opt_default.argtypes = [P]
        L.bsw_extend_seeds.argtypes = [P, P, P, ctypes.c_int64, P, P, P, P, ctypes.c_int32, P]
        L.bsw_ext_last_stats.argtypes = [P, P]
        L.bsw_ksw_align2.argtypes = [P, P, P, P, ctypes.c_int32, P]
        L.bsw_ksw_align2_device.argtypes = [P, P, P, P, ctypes.c_int32, P, P]
        L.bsw_mate_last_stats.argtypes = [P, P]
        L.bsw_ksw_global2.argtypes = [P, P, P, P, ctypes.c_int32, P, ctypes.c_int32, P]
        L.bsw_ksw_global2_device.argtypes = [P, P, P, P, ctypes.c_int32, P, ctypes.c_int32, P, P]
        L.bsw_global_last_stats.argtypes = [P, P]
        L.bsw_set_reference.argtypes = [P, P, ctypes.c_int64]
        L.bsw_extend_seeds_device.argtypes = [P, P, P, P, P, P, ctypes.c_int32, P, P]
        L.bsw_set_option.argtypes = [P, ctypes.c_int, ctypes.c_int64]
        L.bsw_split_by_cells.argtypes = [P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, P]
        L.bsw_chain2aln.argtypes = [P, P, P, ctypes.c_int64, P, P, P, ctypes.c_int32, P, P, P, ctypes.c_int32, P, P]
        L.bsw_chain2aln_device.argtypes = [P, P, P, P, P, ctypes.c_int32, P, P, P, ctypes.c_int32, P, P]
        L.bsw_chain_last_stats.argtypes = [P, P]
        L.bsw_chain2aln_resident.argtypes = [P, P, P, P, P, ctypes.c_int32, P, P, P, ctypes.c_int32, P, P]
        L.bsw_chain2aln_resident.restype = ctypes.c_int
        L.bsw_mem_opt_default.argtypes = [P]
        L.bsw_fmi_build.argtypes = [P, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(P)]
        L.bsw_fmi_build2.argtypes = [P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(P)]
        L.bsw_fmi_build2.restype = ctypes.c_int
        L.bsw_fmi_check.argtypes = [P, P]
        L.bsw_fmi_check.restype = ctypes.c_int
        L.bsw_fmi_destroy.argtypes = [P]
        L.bsw_fmi_get_info.argtypes = [P, P]
        L.bsw_fmi_copy_sa.argtypes = [P, P]
        L.bsw_fmi_copy_bwt.argtypes = [P, P]
        L.bsw_mem_collect_intv.argtypes = [P, P, P, P, P, ctypes.c_int32, P, ctypes.c_int32, P]
        L.bsw_mem_collect_intv_device.argtypes = [P, P, P, P, P, ctypes.c_int32, ctypes.c_int32, P, ctypes.c_int32,
                                                  P, P]
        L.bsw_fmi_sa_device.argtypes = [P, P, ctypes.c_int64, P, P]
        L.bsw_fmi_last_kernel_ms.argtypes = [P, P]
        L.bsw_chain_opt_default.argtypes = [P]
        L.bsw_mem_chain_device.argtypes = [P, P, P, ctypes.c_int32, P, ctypes.c_int32, P, P, P, P, ctypes.c_int64,
                                           P, P]
        L.bsw_mem_chain_device.restype = ctypes.c_int
        L.bsw_pack_batch.argtypes = [P, P, P, ctypes.c_int32, P, ctypes.c_int64, P]
        L.bsw_get_scores_packed_device.argtypes = [P, P, P, ctypes.c_int32, ctypes.c_int, P, P]
        for f in ("bsw_create", "bsw_create_on", "bsw_get_scores", "bsw_get_scores_device", "bsw_last_stats",
                  "bsw_pack_batch", "bsw_get_scores_packed_device",
                  "bsw_abi_version", "bsw_extend_seeds", "bsw_ext_last_stats", "bswb_write",
                  "bswb_read_header", "bswb_read", "bsw_ksw_align2", "bsw_ksw_align2_device",
                  "bsw_mate_last_stats", "bsw_ksw_global2", "bsw_ksw_global2_device", "bsw_global_last_stats",
                  "bsw_set_reference", "bsw_extend_seeds_device", "bsw_set_option",
               "bsw_split_by_cells", "bsw_chain2aln", "bsw_chain2aln_device", "bsw_chain_last_stats",
                  "bsw_fmi_build", "bsw_fmi_get_info", "bsw_fmi_copy_sa", "bsw_fmi_copy_bwt", "bsw_mem_collect_intv",
                  "bsw_mem_collect_intv_device", "bsw_fmi_sa_device", "bsw_fmi_last_kernel_ms"):
            getattr(L, f).restype = ctypes.c_int
        _hip = L
    return _hip


def _check(rc):
    if rc != 0:
        raise BswError(f"bsw error {rc}: {hip_lib().bsw_strerror(rc).decode()}")


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


class Engine:
    """Python mirror of the C++ shim: one engine = one bsw_ctx_t."""

    def __init__(self, params: Params | None = None, device: int = 0, n_gpus: int = 1,
                 devices: list[int] | None = None, **options):
        """devices: explicit logical-device -> HIP-device map (bsw_create_on; repeats allowed,
        the rehearsal of an n-GPU context on a smaller box); else devices [device, device + n_gpus)."""
        self.params = params if params is not None else default_params()
        self._ctx = ctypes.c_void_p()
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*devices)
            _check(hip_lib().bsw_create_on(ctypes.byref(self.params), arr, len(devices), ctypes.byref(self._ctx)))
        else:
            _check(hip_lib().bsw_create(ctypes.byref(self.params), device, n_gpus, ctypes.byref(self._ctx)))
        for k, v in options.items():
            self.set_option(k, v)

    _OPTS = {"kernel8": OPT_KERNEL8, "fork": OPT_FORK, "sortkey": OPT_SORTKEY, "glob_band": OPT_GLOB_BAND,
             "ext_chunk": OPT_EXT_CHUNK, "host_chunk": OPT_HOST_CHUNK, "long": OPT_LONG, "host_pack": OPT_HOST_PACK,
             "small_batch": OPT_SMALL_BATCH, "split_min": OPT_SPLIT_MIN, "coalesce": OPT_COALESCE, "coalesce_leaders": OPT_COALESCE_LEADERS, "group_kernel": OPT_GROUP_KERNEL, "mid_batch": OPT_MID_BATCH,
             "coalesce_linger": OPT_COALESCE_LINGER, "gq32_max": OPT_GQ32_MAX,
             "test_misroute": OPT_TEST_MISROUTE, "test_fail_alloc": OPT_TEST_FAIL_ALLOC}

    def set_option(self, name, value: int):
        """bsw_set_option by name (kernel8, fork, sortkey, glob_band, ext_chunk, host_chunk, test_misroute)
        or by BSW_OPT_* number."""
        opt = self._OPTS[name] if isinstance(name, str) else int(name)
        _check(hip_lib().bsw_set_option(self._ctx, opt, int(value)))

    def close(self):
        if self._ctx:
            hip_lib().bsw_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def get_scores(self, pairs: np.ndarray, ref: np.ndarray, qer: np.ndarray, w: int,
                   cell_bits: int = 16):
        """getScores16 / getScores8 on host buffers; results in place in `pairs`."""
        assert pairs.dtype == SEQPAIR_DTYPE and pairs.flags.c_contiguous
        ref = np.ascontiguousarray(ref, dtype=np.uint8)
        qer = np.ascontiguousarray(qer, dtype=np.uint8)
        _check(hip_lib().bsw_get_scores(self._ctx, _ptr(pairs), _ptr(ref), _ptr(qer),
                                        len(pairs), w, cell_bits))

    def get_scores_device(self, d_pairs: int, d_ref: int, d_qer: int, n: int, w: int,
                          cell_bits: int = 16, stream: int = 0):
        """Device-resident call: raw device pointers (e.g. torch tensor .data_ptr())."""
        _check(hip_lib().bsw_get_scores_device(self._ctx, ctypes.c_void_p(d_pairs),
                                               ctypes.c_void_p(d_ref), ctypes.c_void_p(d_qer),
                                               n, w, cell_bits, ctypes.c_void_p(stream)))

    def get_scores_packed_device(self, d_packed: int, desc: "Packed", w: int, cell_bits: int, d_out: int,
                                 stream: int = 0):
        """bsw_get_scores_packed_device: a packed batch (bsw_pack_batch) resident at d_packed;
        the 6 output int32 per pair go to d_out."""
        _check(hip_lib().bsw_get_scores_packed_device(self._ctx, ctypes.c_void_p(d_packed), ctypes.byref(desc), w,
                                                      cell_bits, ctypes.c_void_p(d_out), ctypes.c_void_p(stream)))

    def last_stats(self) -> Stats:
        s = Stats()
        _check(hip_lib().bsw_last_stats(self._ctx, ctypes.byref(s)))
        return s


class Packed(ctypes.Structure):
    """bsw_packed_t: descriptor of a batch in the 2-bit wire form (bsw_pack_batch)"""
    _fields_ = [("n", ctypes.c_int32), ("n_exc_ref", ctypes.c_int32), ("n_exc_qer", ctypes.c_int32),
                ("pad_", ctypes.c_int32), ("ref_bytes", ctypes.c_int64), ("qer_bytes", ctypes.c_int64),
                ("rec_off", ctypes.c_int64), ("ref_off", ctypes.c_int64), ("qer_off", ctypes.c_int64),
                ("exc_off", ctypes.c_int64), ("total_bytes", ctypes.c_int64)]
    FIELDS = ("n", "n_exc_ref", "n_exc_qer", "ref_bytes", "qer_bytes", "rec_off", "ref_off", "qer_off", "exc_off",
              "total_bytes")

    def to_row(self) -> np.ndarray:
        return np.array([getattr(self, f) for f in self.FIELDS], dtype=np.int64)

    @classmethod
    def from_row(cls, row) -> "Packed":
        d = cls()
        for f, v in zip(cls.FIELDS, row):
            setattr(d, f, int(v))
        return d


def pack_batch(pairs: np.ndarray, ref: np.ndarray, qer: np.ndarray, pad_to: int = 0):
    """bsw_pack_batch: (uint8 buffer, Packed) -- the 2-bit wire form of pairs over ref / qer,
    zero-padded to pad_to bytes when that is larger (host-only, no device needed)."""
    assert pairs.dtype == SEQPAIR_DTYPE and pairs.flags.c_contiguous
    ref = np.ascontiguousarray(ref, dtype=np.uint8)
    qer = np.ascontiguousarray(qer, dtype=np.uint8)
    d = Packed()
    L = hip_lib()
    _check(L.bsw_pack_batch(_ptr(pairs), _ptr(ref), _ptr(qer), len(pairs), None, 0, ctypes.byref(d)))
    buf = np.zeros(max(int(d.total_bytes), int(pad_to), 64), dtype=np.uint8)
    _check(L.bsw_pack_batch(_ptr(pairs), _ptr(ref), _ptr(qer), len(pairs), _ptr(buf), len(buf), ctypes.byref(d)))
    return buf, d


def split_by_cells(pairs: np.ndarray, w: int, parts: int) -> np.ndarray:
    """bsw_split_by_cells: parts + 1 cut points of equal static band cells (host-only)."""
    assert pairs.dtype == SEQPAIR_DTYPE and pairs.flags.c_contiguous
    cut = np.zeros(parts + 1, dtype=np.int32)
    _check(hip_lib().bsw_split_by_cells(_ptr(pairs), len(pairs), w, parts, _ptr(cut)))
    return cut


# ---------------------------------------------------------------- .bswb batch files
class BswbHeader(ctypes.Structure):
    """Mirror of bswb_header_t (include/bsw_batch.h), 128 bytes."""
    _fields_ = [("magic", ctypes.c_uint32), ("version", ctypes.c_uint32), ("header_bytes", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("n_pairs", ctypes.c_int64), ("ref_bytes", ctypes.c_int64),
                ("qer_bytes", ctypes.c_int64), ("checksum", ctypes.c_uint64), ("w", ctypes.c_int32),
                ("cell_bits", ctypes.c_int32), ("params", Params), ("reserved", ctypes.c_uint8 * 20)]


def write_batch(path: str, pairs, ref, qer, w: int, cell_bits: int = 16, params=None,
                has_outputs: bool = True):
    """bswb_write: record a batch (+ outputs) for replay."""
    params = params if params is not None else default_params()
    pairs = np.ascontiguousarray(pairs, dtype=SEQPAIR_DTYPE)
    ref = np.ascontiguousarray(ref, dtype=np.uint8)
    qer = np.ascontiguousarray(qer, dtype=np.uint8)
    _check(hip_lib().bswb_write(path.encode(), ctypes.byref(params), w, cell_bits, int(has_outputs),
                                _ptr(pairs), len(pairs), _ptr(ref), len(ref), _ptr(qer), len(qer)))


def read_batch(path: str):
    """bswb_read: (header, pairs, ref, qer); raises BswError on a bad / corrupted file."""
    h = BswbHeader()
    _check(hip_lib().bswb_read_header(path.encode(), ctypes.byref(h)))
    pairs = np.zeros(h.n_pairs, dtype=SEQPAIR_DTYPE)
    ref = np.zeros(max(1, h.ref_bytes), dtype=np.uint8)
    qer = np.zeros(max(1, h.qer_bytes), dtype=np.uint8)
    _check(hip_lib().bswb_read(path.encode(), ctypes.byref(h), _ptr(pairs), _ptr(ref), _ptr(qer)))
    return h, pairs, ref, qer


# ---------------------------------------------------------------- extension pipeline
class ExtOpt(ctypes.Structure):
    """Mirror of bsw_ext_opt_t (include/bsw_ext.h)."""
    _fields_ = [("w", ctypes.c_int32), ("pen_clip5", ctypes.c_int32), ("pen_clip3", ctypes.c_int32),
                ("max_band_try", ctypes.c_int32), ("l_pac", ctypes.c_int64)]


class ExtStats(ctypes.Structure):
    _fields_ = [("n_pairs", ctypes.c_int32 * 4), ("kernel_ms", ctypes.c_float), ("build_ms", ctypes.c_float),
                ("engine_ms", ctypes.c_float), ("interp_ms", ctypes.c_float)]


def ext_opt(**kw) -> ExtOpt:
    o = ExtOpt()
    hip_lib().bsw_ext_opt_default(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def extend_seeds(engine, ref, reads, read_off, read_len, seeds, opt: ExtOpt | None = None):
    """bsw_extend_seeds: one seed per read -> ALNREG_DTYPE regions (local / to-end ends)."""
    opt = opt if opt is not None else ext_opt()
    ref = np.ascontiguousarray(ref, dtype=np.uint8)
    reads = np.ascontiguousarray(reads, dtype=np.uint8)
    read_off = np.ascontiguousarray(read_off, dtype=np.int64)
    read_len = np.ascontiguousarray(read_len, dtype=np.int32)
    seeds = np.ascontiguousarray(seeds, dtype=SEED_DTYPE)
    out = np.zeros(len(seeds), dtype=ALNREG_DTYPE)
    _check(hip_lib().bsw_extend_seeds(engine._ctx, ctypes.byref(opt), _ptr(ref), len(ref), _ptr(reads),
                                      _ptr(read_off), _ptr(read_len), _ptr(seeds), len(seeds), _ptr(out)))
    return out


def set_reference(engine, ref: np.ndarray):
    """bsw_set_reference: keep ref resident in HBM (for extend_seeds_device)."""
    ref = np.ascontiguousarray(ref, dtype=np.uint8)
    _check(hip_lib().bsw_set_reference(engine._ctx, _ptr(ref), len(ref)))


def extend_seeds_device(engine, d_reads: int, d_off: int, d_len: int, d_seeds: int, n: int, d_out: int,
                        opt: ExtOpt | None = None, stream: int = 0):
    """bsw_extend_seeds_device on raw device pointers (resident reference required)."""
    opt = opt if opt is not None else ext_opt()
    V = ctypes.c_void_p
    _check(hip_lib().bsw_extend_seeds_device(engine._ctx, ctypes.byref(opt), V(d_reads), V(d_off), V(d_len),
                                             V(d_seeds), n, V(d_out), V(stream or None)))


def extend_seeds_resident(engine, reads, read_off, read_len, seeds, opt: ExtOpt | None = None):
    """Upload reads / seeds, run bsw_extend_seeds_device against the resident reference, download
    the regions (ALNREG_DTYPE)."""
    import hiprt
    bufs = [hiprt.DeviceBuffer.from_array(np.ascontiguousarray(a, dtype=dt)) for a, dt in
            ((reads, np.uint8), (read_off, np.int64), (read_len, np.int32), (seeds, SEED_DTYPE))]
    out = np.zeros(len(seeds), dtype=ALNREG_DTYPE)
    d_out = hiprt.DeviceBuffer(out.nbytes)
    extend_seeds_device(engine, bufs[0].ptr, bufs[1].ptr, bufs[2].ptr, bufs[3].ptr, len(seeds), d_out.ptr, opt)
    d_out.download(out)
    return out


def ext_last_stats(engine) -> ExtStats:
    s = ExtStats()
    _check(hip_lib().bsw_ext_last_stats(engine._ctx, ctypes.byref(s)))
    return s


# ---------------------------------------------------------------- mate rescue (bsw_mate.h)
class MateStats(ctypes.Structure):
    _fields_ = [("fwd_ms", ctypes.c_float), ("rev_ms", ctypes.c_float), ("n_fwd", ctypes.c_int32),
                ("n_rev", ctypes.c_int32), ("cells_fwd", ctypes.c_int64)]


def ksw_align2(engine, pairs: np.ndarray, ref: np.ndarray, qer: np.ndarray) -> np.ndarray:
    """bsw_ksw_align2: per SeqPair (len1 = target, len2 = query, h0 = xtra) upstream
    ksw_align2's kswr_t -> KSWR_DTYPE array."""
    assert pairs.dtype == SEQPAIR_DTYPE and pairs.flags.c_contiguous
    ref = np.ascontiguousarray(ref, dtype=np.uint8)
    qer = np.ascontiguousarray(qer, dtype=np.uint8)
    out = np.zeros(len(pairs), dtype=KSWR_DTYPE)
    _check(hip_lib().bsw_ksw_align2(engine._ctx, _ptr(pairs), _ptr(ref), _ptr(qer), len(pairs), _ptr(out)))
    return out


def ksw_align2_device(engine, d_pairs: int, d_ref: int, d_qer: int, n: int, d_aln: int, stream: int = 0):
    _check(hip_lib().bsw_ksw_align2_device(engine._ctx, ctypes.c_void_p(d_pairs), ctypes.c_void_p(d_ref),
                                           ctypes.c_void_p(d_qer), n, ctypes.c_void_p(d_aln),
                                           ctypes.c_void_p(stream or None)))


def mate_last_stats(engine) -> MateStats:
    s = MateStats()
    _check(hip_lib().bsw_mate_last_stats(engine._ctx, ctypes.byref(s)))
    return s


class GlobalStats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_float), ("n_jobs", ctypes.c_int32), ("n_lane", ctypes.c_int32),
                ("n_wide", ctypes.c_int32), ("n_launches", ctypes.c_int32), ("cells", ctypes.c_int64),
                ("z_bytes", ctypes.c_int64), ("n_tb_retry", ctypes.c_int32), ("pad_", ctypes.c_int32)]


def ksw_global2(engine, pairs: np.ndarray, ref: np.ndarray, qer: np.ndarray, stride: int = 64):
    """bsw_ksw_global2 (include/bsw_global.h): per SeqPair (len1 = target, len2 = query, h0 = w)
    upstream ksw_global2 -> (score, cigar[n, stride] uint32 or None, n_cigar); scores are also
    written into pairs['score']."""
    assert pairs.dtype == SEQPAIR_DTYPE and pairs.flags.c_contiguous
    ref = np.ascontiguousarray(ref, dtype=np.uint8)
    qer = np.ascontiguousarray(qer, dtype=np.uint8)
    n = len(pairs)
    cig = np.zeros((n, stride), dtype=np.uint32) if stride > 0 else None
    ncig = np.zeros(n, dtype=np.int32)
    _check(hip_lib().bsw_ksw_global2(engine._ctx, _ptr(pairs), _ptr(ref), _ptr(qer), n,
                                     _ptr(cig) if cig is not None else None, stride, _ptr(ncig)))
    return pairs["score"].copy(), cig, ncig


def ksw_global2_device(engine, d_pairs: int, d_ref: int, d_qer: int, n: int, d_cigar: int, stride: int,
                       d_ncig: int, stream: int = 0):
    _check(hip_lib().bsw_ksw_global2_device(engine._ctx, ctypes.c_void_p(d_pairs), ctypes.c_void_p(d_ref),
                                            ctypes.c_void_p(d_qer), n, ctypes.c_void_p(d_cigar or None),
                                            stride, ctypes.c_void_p(d_ncig or None),
                                            ctypes.c_void_p(stream or None)))


def global_last_stats(engine) -> GlobalStats:
    s = GlobalStats()
    _check(hip_lib().bsw_global_last_stats(engine._ctx, ctypes.byref(s)))
    return s


# ---------------------------------------------------------------- synthetic batches
class SynthCfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("tlen", ctypes.c_int32), ("qlen", ctypes.c_int32),
                ("h0_lo", ctypes.c_int32), ("h0_hi", ctypes.c_int32),
                ("p_sub", ctypes.c_double), ("p_indel", ctypes.c_double),
                ("p_unrelated", ctypes.c_double), ("p_n", ctypes.c_double)]


_synth = None


def synth_lib():
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_LIB):
            raise BswError(f"{SYNTH_LIB} not built: run `make synth`")
        L = ctypes.CDLL(SYNTH_LIB)
        L.bsw_synth_default.argtypes = [ctypes.c_void_p]
        L.bsw_synth_batch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.bsw_synth_reference.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p]
        L.bsw_reads_default.argtypes = [ctypes.c_void_p]
        L.bsw_synth_reads.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.bsw_synth_reads.restype = ctypes.c_int32
        L.bsw_synth_pe_seeds.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_double,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.bsw_synth_pe_seeds.restype = ctypes.c_int32
        L.bsw_mates_default.argtypes = [ctypes.c_void_p]
        L.bsw_synth_mates.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
        L.bsw_synth_mates.restype = ctypes.c_int32
        L.bsw_globals_default.argtypes = [ctypes.c_void_p]
        L.bsw_synth_globals.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
        L.bsw_synth_globals.restype = ctypes.c_int32
        _synth = L
    return _synth


def synth_cfg(**kw) -> SynthCfg:
    c = SynthCfg()
    synth_lib().bsw_synth_default(ctypes.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def synth_batch(n: int, pair_base: int = 0, cfg: SynthCfg | None = None):
    """C2 workload batch: (pairs, ref, qer) numpy arrays in the upstream layout."""
    cfg = cfg if cfg is not None else synth_cfg()
    pairs = np.zeros(n, dtype=SEQPAIR_DTYPE)
    ref = np.zeros(max(1, n * cfg.tlen), dtype=np.uint8)
    qer = np.zeros(max(1, n * cfg.qlen), dtype=np.uint8)
    synth_lib().bsw_synth_batch(ctypes.byref(cfg), pair_base, n, _ptr(pairs), _ptr(ref),
                                _ptr(qer))
    return pairs, ref, qer


class ReadsCfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("read_len", ctypes.c_int32), ("min_seed", ctypes.c_int32),
                ("p_sub", ctypes.c_double), ("p_indel", ctypes.c_double), ("p_unrelated", ctypes.c_double)]


def reads_cfg(**kw) -> ReadsCfg:
    c = ReadsCfg()
    synth_lib().bsw_reads_default(ctypes.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def synth_reference(length: int, seed: int = 7, p_n: float = 0.0005) -> np.ndarray:
    """Random reference (codes 0..3, N = 4 at rate p_n), reproducible per seed."""
    ref = np.empty(length, dtype=np.uint8)
    synth_lib().bsw_synth_reference(seed, length, p_n, _ptr(ref))
    return ref


def synth_reads(ref: np.ndarray, n: int, read_base: int = 0, cfg: ReadsCfg | None = None):
    """Reads sampled from ref with one exact seed each: (reads, read_off, read_len, seeds, origin)."""
    cfg = cfg if cfg is not None else reads_cfg()
    L = cfg.read_len
    reads = np.zeros(max(1, n * L), dtype=np.uint8)
    seeds = np.zeros(n, dtype=SEED_DTYPE)
    origin = np.zeros(n, dtype=np.int64)
    r = synth_lib().bsw_synth_reads(ctypes.byref(cfg), _ptr(ref), len(ref), read_base, n, _ptr(reads),
                                    _ptr(seeds), _ptr(origin))
    if r < 0:
        raise BswError("bsw_synth_reads: reference too short for the read length")
    read_off = np.arange(n, dtype=np.int64) * L
    read_len = np.full(n, L, dtype=np.int32)
    return reads, read_off, read_len, seeds, origin


def synth_pe_seeds(ref: np.ndarray, n_pairs: int, pair_base: int = 0, cfg: ReadsCfg | None = None,
                   ins=(400, 600), p_spurious: float = 0.1):
    """Paired-end reads with several seeds each (bsw_synth_pe_seeds): (reads, read_off, read_len,
    seeds, seed_read, seed_chain); read_off / read_len are PER READ (2 n_pairs reads; reads 2k /
    2k+1 are the mates of fragment k), seed_read / seed_chain map each seed to its read and chain
    (bsw_chain2aln's input layout; for bsw_extend_seeds index read_off by seed_read)."""
    cfg = cfg if cfg is not None else reads_cfg()
    L = cfg.read_len
    n_reads = 2 * n_pairs
    reads = np.zeros(max(1, n_reads * L), dtype=np.uint8)
    seeds = np.zeros(max(1, n_reads * 9), dtype=SEED_DTYPE)
    seed_read = np.zeros(max(1, n_reads * 9), dtype=np.int32)
    seed_chain = np.zeros(max(1, n_reads * 9), dtype=np.int32)
    ns = synth_lib().bsw_synth_pe_seeds(ctypes.byref(cfg), _ptr(ref), len(ref), pair_base, n_pairs, ins[0], ins[1],
                                        ctypes.c_double(p_spurious), _ptr(reads), _ptr(seeds), _ptr(seed_read),
                                        _ptr(seed_chain))
    if ns < 0:
        raise BswError("bsw_synth_pe_seeds: reference too short")
    read_off = np.arange(n_reads, dtype=np.int64) * L
    read_len = np.full(n_reads, L, dtype=np.int32)
    return reads, read_off, read_len, seeds[:ns].copy(), seed_read[:ns].copy(), seed_chain[:ns].copy()


class ChainStats(ctypes.Structure):
    _fields_ = [("rounds", ctypes.c_int32), ("n_extended", ctypes.c_int32), ("n_skipped", ctypes.c_int32),
                ("n_pairs", ctypes.c_int32 * 4), ("kernel_ms", ctypes.c_float), ("ext_ms", ctypes.c_float),
                ("check_ms", ctypes.c_float), ("prep_ms", ctypes.c_float)]


def chain2aln(engine, ref, reads, read_off, read_len, seeds, seed_read, seed_chain, opt: ExtOpt | None = None):
    """bsw_chain2aln: (regions per seed, extended flags)."""
    opt = opt if opt is not None else ext_opt()
    ref = np.ascontiguousarray(ref, dtype=np.uint8)
    reads = np.ascontiguousarray(reads, dtype=np.uint8)
    read_off = np.ascontiguousarray(read_off, dtype=np.int64)
    read_len = np.ascontiguousarray(read_len, dtype=np.int32)
    seeds = np.ascontiguousarray(seeds, dtype=SEED_DTYPE)
    seed_read = np.ascontiguousarray(seed_read, dtype=np.int32)
    seed_chain = np.ascontiguousarray(seed_chain, dtype=np.int32)
    out = np.zeros(len(seeds), dtype=ALNREG_DTYPE)
    ext = np.zeros(len(seeds), dtype=np.int32)
    _check(hip_lib().bsw_chain2aln(engine._ctx, ctypes.byref(opt), _ptr(ref), len(ref), _ptr(reads), _ptr(read_off),
                                   _ptr(read_len), len(read_len), _ptr(seeds), _ptr(seed_read), _ptr(seed_chain),
                                   len(seeds), _ptr(out), _ptr(ext)))
    return out, ext


def chain2aln_device(engine, d_reads: int, read_off, read_len, seeds, seed_read, seed_chain,
                     opt: ExtOpt | None = None, out=None, ext=None):
    """bsw_chain2aln_device: reads resident at d_reads (device pointer), reference resident;
    `out` / `ext` may be preallocated (ALNREG_DTYPE / int32, len(seeds))."""
    opt = opt if opt is not None else ext_opt()
    read_off = np.ascontiguousarray(read_off, dtype=np.int64)
    read_len = np.ascontiguousarray(read_len, dtype=np.int32)
    seeds = np.ascontiguousarray(seeds, dtype=SEED_DTYPE)
    seed_read = np.ascontiguousarray(seed_read, dtype=np.int32)
    seed_chain = np.ascontiguousarray(seed_chain, dtype=np.int32)
    out = np.zeros(len(seeds), dtype=ALNREG_DTYPE) if out is None else out
    ext = np.zeros(len(seeds), dtype=np.int32) if ext is None else ext
    assert out.dtype == ALNREG_DTYPE and len(out) == len(seeds) and ext.dtype == np.int32 and len(ext) == len(seeds)
    _check(hip_lib().bsw_chain2aln_device(engine._ctx, ctypes.byref(opt), ctypes.c_void_p(d_reads), _ptr(read_off),
                                          _ptr(read_len), len(read_len), _ptr(seeds), _ptr(seed_read),
                                          _ptr(seed_chain), len(seeds), _ptr(out), _ptr(ext)))
    return out, ext


def chain2aln_resident(engine, d_reads: int, d_off: int, d_len: int, n_reads: int, d_seeds: int, d_sr: int,
                       d_sc: int, n_seeds: int, d_out: int, d_ext: int, opt: ExtOpt | None = None):
    """bsw_chain2aln_resident: every array a device pointer (regions / flags into d_out / d_ext)."""
    opt = opt if opt is not None else ext_opt()
    V = ctypes.c_void_p
    _check(hip_lib().bsw_chain2aln_resident(engine._ctx, ctypes.byref(opt), V(d_reads), V(d_off), V(d_len), n_reads,
                                            V(d_seeds), V(d_sr), V(d_sc), n_seeds, V(d_out), V(d_ext)))


def chain_last_stats(engine) -> ChainStats:
    st = ChainStats()
    _check(hip_lib().bsw_chain_last_stats(engine._ctx, ctypes.byref(st)))
    return st


class MatesCfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("read_len", ctypes.c_int32), ("win_len", ctypes.c_int32),
                ("a", ctypes.c_int32), ("min_seed", ctypes.c_int32), ("p_true", ctypes.c_double),
                ("p_sub", ctypes.c_double), ("p_indel", ctypes.c_double)]


def mates_cfg(**kw) -> MatesCfg:
    c = MatesCfg()
    synth_lib().bsw_mates_default(ctypes.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def synth_mates(ref: np.ndarray, n: int, base: int = 0, cfg: MatesCfg | None = None):
    """Mate-rescue jobs against ref (bsw_synth_mates): (pairs, qer); seqBufRef is ref itself."""
    cfg = cfg if cfg is not None else mates_cfg()
    pairs = np.zeros(n, dtype=SEQPAIR_DTYPE)
    qer = np.zeros(max(1, n * cfg.read_len), dtype=np.uint8)
    r = synth_lib().bsw_synth_mates(ctypes.byref(cfg), _ptr(ref), len(ref), base, n, _ptr(pairs), _ptr(qer))
    if r < 0:
        raise BswError("bsw_synth_mates: reference too short for the window")
    return pairs, qer


class GlobalsCfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("read_len", ctypes.c_int32), ("w_cap", ctypes.c_int32),
                ("a", ctypes.c_int32), ("o_del", ctypes.c_int32), ("e_del", ctypes.c_int32),
                ("o_ins", ctypes.c_int32), ("e_ins", ctypes.c_int32), ("p_sub", ctypes.c_double),
                ("p_indel", ctypes.c_double)]


def globals_cfg(**kw) -> GlobalsCfg:
    c = GlobalsCfg()
    synth_lib().bsw_globals_default(ctypes.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def synth_globals(ref: np.ndarray, n: int, base: int = 0, cfg: GlobalsCfg | None = None):
    """ksw_global2 jobs shaped like bwa_gen_cigar2's (bsw_synth_globals): (pairs, qer); seqBufRef
    is ref itself, h0 = the band w."""
    cfg = cfg if cfg is not None else globals_cfg()
    pairs = np.zeros(n, dtype=SEQPAIR_DTYPE)
    qer = np.zeros(max(1, n * cfg.read_len), dtype=np.uint8)
    r = synth_lib().bsw_synth_globals(ctypes.byref(cfg), _ptr(ref), len(ref), base, n, _ptr(pairs), _ptr(qer))
    if r < 0:
        raise BswError("bsw_synth_globals: reference too short for the read length")
    return pairs, qer


# ---- include/bsw_fmi.h: FM-index SMEM seeding

BWTINTV_DTYPE = np.dtype([("k", "<u8"), ("l", "<u8"), ("s", "<u8"), ("info", "<u8")])   # bsw_bwtintv_t
assert BWTINTV_DTYPE.itemsize == 32


class MemOpt(ctypes.Structure):
    _fields_ = [("min_seed_len", ctypes.c_int32), ("split_width", ctypes.c_int32),
                ("max_mem_intv", ctypes.c_int32), ("split_factor", ctypes.c_float)]


class FmiInfo(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("sentinel", ctypes.c_int64), ("count", ctypes.c_int64 * 5),
                ("device_bytes", ctypes.c_int64), ("build_s", ctypes.c_float)]


def mem_opt(**kw) -> MemOpt:
    o = MemOpt()
    hip_lib().bsw_mem_opt_default(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


FMI_GPU_BUILD, FMI_WIDE, FMI_NO_TEXT, FMI_PLAIN_ENT = 1, 2, 4, 8


class Fmi:
    """One resident FM-index (bsw_fmi_t) of ref + reverse-complement(ref) on `device`;
    flags: FMI_GPU_BUILD / FMI_WIDE / FMI_NO_TEXT (bsw_fmi_build2), None: the library's choice."""

    def __init__(self, ref: np.ndarray, device: int = 0, flags: int | None = None):
        self.ref = np.ascontiguousarray(ref, dtype=np.uint8)
        self._f = ctypes.c_void_p()
        if flags is None:
            _check(hip_lib().bsw_fmi_build(_ptr(self.ref), len(self.ref), device, ctypes.byref(self._f)))
        else:
            _check(hip_lib().bsw_fmi_build2(_ptr(self.ref), len(self.ref), device, flags, ctypes.byref(self._f)))

    def close(self):
        if self._f:
            hip_lib().bsw_fmi_destroy(self._f)
            self._f = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self) -> int:
        """bsw_fmi_check: number of violated index invariants (0 = consistent)"""
        bad = ctypes.c_int64(-1)
        _check(hip_lib().bsw_fmi_check(self._f, ctypes.byref(bad)))
        return bad.value

    def info(self) -> FmiInfo:
        i = FmiInfo()
        _check(hip_lib().bsw_fmi_get_info(self._f, ctypes.byref(i)))
        return i

    def sa(self) -> np.ndarray:
        a = np.zeros(self.info().n + 1, dtype=np.int64)
        _check(hip_lib().bsw_fmi_copy_sa(self._f, _ptr(a)))
        return a

    def bwt(self) -> np.ndarray:
        a = np.zeros(self.info().n + 1, dtype=np.uint8)
        _check(hip_lib().bsw_fmi_copy_bwt(self._f, _ptr(a)))
        return a

    def collect_intv(self, reads, read_off, read_len, cap: int = 256, opt: MemOpt | None = None, strict=True):
        """bsw_mem_collect_intv (host buffers) -> (intervals [n, cap], counts [n])"""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        read_off = np.ascontiguousarray(read_off, dtype=np.int64)
        read_len = np.ascontiguousarray(read_len, dtype=np.int32)
        n = len(read_len)
        out = np.zeros((n, cap), dtype=BWTINTV_DTYPE)
        cnt = np.zeros(n, dtype=np.int32)
        o = opt if opt is not None else mem_opt()
        rc = hip_lib().bsw_mem_collect_intv(self._f, ctypes.byref(o), _ptr(reads), _ptr(read_off), _ptr(read_len),
                                            n, _ptr(out), cap, _ptr(cnt))
        if strict or rc != -34:
            _check(rc)
        return out, cnt

    def collect_intv_device(self, d_reads: int, d_off: int, d_len: int, n: int, max_len: int, d_mems: int, cap: int,
                            d_cnt: int, opt: MemOpt | None = None, stream: int = 0) -> int:
        o = opt if opt is not None else mem_opt()
        return hip_lib().bsw_mem_collect_intv_device(self._f, ctypes.byref(o), ctypes.c_void_p(d_reads),
                                                     ctypes.c_void_p(d_off), ctypes.c_void_p(d_len), n, max_len,
                                                     ctypes.c_void_p(d_mems), cap, ctypes.c_void_p(d_cnt),
                                                     ctypes.c_void_p(stream or None))

    def sa_device(self, d_k: int, n: int, d_pos: int, stream: int = 0):
        _check(hip_lib().bsw_fmi_sa_device(self._f, ctypes.c_void_p(d_k), n, ctypes.c_void_p(d_pos),
                                           ctypes.c_void_p(stream or None)))

    def last_kernel_ms(self) -> float:
        v = ctypes.c_float()
        _check(hip_lib().bsw_fmi_last_kernel_ms(self._f, ctypes.byref(v)))
        return v.value

    def mem_chain_device(self, d_len: int, n: int, d_mems: int, cap: int, d_cnt: int, d_seeds: int, d_sr: int,
                         d_sc: int, seed_cap: int, opt: "ChainOpt | None" = None, stream: int = 0):
        """bsw_mem_chain_device -> (status, seeds needed / written)"""
        o = opt if opt is not None else chain_opt()
        ns = ctypes.c_int64(0)
        rc = hip_lib().bsw_mem_chain_device(self._f, ctypes.byref(o), ctypes.c_void_p(d_len), n,
                                            ctypes.c_void_p(d_mems), cap, ctypes.c_void_p(d_cnt),
                                            ctypes.c_void_p(d_seeds or None), ctypes.c_void_p(d_sr or None),
                                            ctypes.c_void_p(d_sc or None), seed_cap, ctypes.byref(ns),
                                            ctypes.c_void_p(stream or None))
        return rc, ns.value


class ChainOpt(ctypes.Structure):
    """Mirror of bsw_chain_opt_t (include/bsw_fmi.h)."""
    _fields_ = [("max_occ", ctypes.c_int32), ("w", ctypes.c_int32), ("max_chain_gap", ctypes.c_int32),
                ("min_chain_weight", ctypes.c_int32), ("min_seed_len", ctypes.c_int32),
                ("max_chain_extend", ctypes.c_int32), ("drop_ratio", ctypes.c_float), ("mask_level", ctypes.c_float)]


def chain_opt(**kw) -> ChainOpt:
    o = ChainOpt()
    hip_lib().bsw_chain_opt_default(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def seed_and_chain(fmi: Fmi, d_reads, read_off, read_len, cap: int = 256, mopt=None, copt=None):
    """The GPU seeding front end of mem_align1_core over resident reads: bsw_mem_collect_intv_device
    -> bsw_mem_chain_device.  d_reads: a hiprt.DeviceBuffer of the reads.  Returns host copies
    (seeds, seed_read, seed_chain) and the device buffers holding them (d_seeds, d_sr, d_sc)."""
    import hiprt
    read_off = np.ascontiguousarray(read_off, dtype=np.int64)
    read_len = np.ascontiguousarray(read_len, dtype=np.int32)
    n = len(read_len)
    d_off, d_len = hiprt.DeviceBuffer.from_array(read_off), hiprt.DeviceBuffer.from_array(read_len)
    d_mems = hiprt.DeviceBuffer(max(1, n * cap) * BWTINTV_DTYPE.itemsize)
    d_cnt = hiprt.DeviceBuffer(max(1, n) * 4)
    _check(fmi.collect_intv_device(d_reads.ptr, d_off.ptr, d_len.ptr, n, int(read_len.max(initial=0)), d_mems.ptr, cap,
                                   d_cnt.ptr, mopt))
    rc, need = fmi.mem_chain_device(d_len.ptr, n, d_mems.ptr, cap, d_cnt.ptr, 0, 0, 0, 0, copt)
    if rc not in (0, -34):
        _check(rc)
    d_seeds = hiprt.DeviceBuffer(max(1, need) * SEED_DTYPE.itemsize)
    d_sr, d_sc = hiprt.DeviceBuffer(max(1, need) * 4), hiprt.DeviceBuffer(max(1, need) * 4)
    rc, got = fmi.mem_chain_device(d_len.ptr, n, d_mems.ptr, cap, d_cnt.ptr, d_seeds.ptr, d_sr.ptr, d_sc.ptr, need, copt)
    _check(rc)
    assert got == need
    seeds = d_seeds.download(np.zeros(need, dtype=SEED_DTYPE)) if need else np.zeros(0, SEED_DTYPE)
    sr = d_sr.download(np.zeros(need, dtype=np.int32)) if need else np.zeros(0, np.int32)
    sc = d_sc.download(np.zeros(need, dtype=np.int32)) if need else np.zeros(0, np.int32)
    return (seeds, sr, sc), (d_seeds, d_sr, d_sc), (d_off, d_len)
