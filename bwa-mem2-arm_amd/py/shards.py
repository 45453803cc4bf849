"""Batch scatter / gather over ranks -- BASELINE configs[4]'s "batch scatter" of SeqPair batches.

One batch (SeqPair records + the two byte buffers they index, upstream's layout) is cut into
contiguous pair ranges of equal static band cells (bsw_split_by_cells).  Each
range becomes ONE byte buffer

    [SeqPair x n | ref bytes | qer bytes | zero padding]

with idr / idq rebased to the range's own byte extents, every buffer padded to the largest, so a
single scatter moves every rank's shard and the rank computes on it in place (bsw_get_scores_device
on pointers into the buffer).  Outputs come back as 6 int32 per pair (score, tle, gtle, qle,
gscore, max_off) by one gather.  numpy here: bench.py moves the buffers as torch tensors between
the GPUs (backend "nccl" = RCCL over xGMI), tests/test_dist.py as CPU tensors over gloo."""

import numpy as np

import bsw

OUT_COLS = slice(8, 14)          # int32 columns score .. max_off of a SeqPair (56 B = 14 int32)


def shard_layout(pairs: np.ndarray, cut) -> list:
    """Per range k of `cut`: (lo, hi, r_lo, r_hi, q_lo, q_hi) -- its pairs and the byte extents of
    the ref / qer windows they address (empty windows count as nothing)."""
    out = []
    for k in range(len(cut) - 1):
        lo, hi = int(cut[k]), int(cut[k + 1])
        p = pairs[lo:hi]
        r_has, q_has = p["len1"] > 0, p["len2"] > 0
        r_lo = int(p["idr"][r_has].min()) if r_has.any() else 0
        r_hi = int((p["idr"][r_has].astype(np.int64) + p["len1"][r_has]).max()) if r_has.any() else 0
        q_lo = int(p["idq"][q_has].min()) if q_has.any() else 0
        q_hi = int((p["idq"][q_has].astype(np.int64) + p["len2"][q_has]).max()) if q_has.any() else 0
        out.append((lo, hi, r_lo, r_hi, q_lo, q_hi))
    return out


def shard_meta(layout) -> np.ndarray:
    """(n, ref bytes, qer bytes) per range as int64 [world, 3] (what every rank needs to find its
    records and windows inside its buffer)."""
    return np.array([(hi - lo, r_hi - r_lo, q_hi - q_lo) for lo, hi, r_lo, r_hi, q_lo, q_hi in layout],
                    dtype=np.int64).reshape(-1, 3)


def buffer_bytes(meta: np.ndarray) -> int:
    """Bytes of one padded shard buffer (a multiple of 64)."""
    if len(meta) == 0:
        return 64
    need = int((meta[:, 0] * bsw.SEQPAIR_DTYPE.itemsize + meta[:, 1] + meta[:, 2]).max()) + 8
    return (need + 63) & ~63


def pack_shards(pairs: np.ndarray, ref: np.ndarray, qer: np.ndarray, cut):
    """[world, S] uint8: every range's records (idr / idq rebased) and windows; plus its meta."""
    layout = shard_layout(pairs, cut)
    meta = shard_meta(layout)
    S = buffer_bytes(meta)
    bufs = np.zeros((len(layout), S), dtype=np.uint8)
    for k, (lo, hi, r_lo, r_hi, q_lo, q_hi) in enumerate(layout):
        n = hi - lo
        p = pairs[lo:hi].copy()
        p["idr"] = np.where(p["len1"] > 0, p["idr"] - r_lo, 0)
        p["idq"] = np.where(p["len2"] > 0, p["idq"] - q_lo, 0)
        o = n * bsw.SEQPAIR_DTYPE.itemsize
        bufs[k, :o] = p.view(np.uint8)
        bufs[k, o:o + (r_hi - r_lo)] = ref[r_lo:r_hi]
        bufs[k, o + (r_hi - r_lo):o + (r_hi - r_lo) + (q_hi - q_lo)] = qer[q_lo:q_hi]
    return bufs, meta


def offsets(meta_row) -> tuple:
    """Byte offsets (pairs, ref, qer) inside one shard buffer."""
    n, rb, _ = (int(x) for x in meta_row)
    o = n * bsw.SEQPAIR_DTYPE.itemsize
    return 0, o, o + rb


def unpack_shard(buf: np.ndarray, meta_row):
    """numpy views (pairs, ref, qer) into one shard buffer (computing on them writes the buffer)."""
    n, rb, qb = (int(x) for x in meta_row)
    po, ro, qo = offsets(meta_row)
    pairs = buf[po:po + n * bsw.SEQPAIR_DTYPE.itemsize].view(bsw.SEQPAIR_DTYPE)
    return pairs, buf[ro:ro + rb], buf[qo:qo + qb]


def outputs(pairs: np.ndarray) -> np.ndarray:
    """The 6 output int32 per pair, [n, 6]."""
    return np.ascontiguousarray(pairs.view(np.int32).reshape(-1, 14)[:, OUT_COLS])


def merge_outputs(pairs: np.ndarray, outs, cut) -> None:
    """Write gathered [n_k, 6] output blocks (rank order) back into the whole batch's records."""
    v = pairs.view(np.int32).reshape(-1, 14)
    for k, o in enumerate(outs):
        lo, hi = int(cut[k]), int(cut[k + 1])
        v[lo:hi, OUT_COLS] = np.asarray(o)[:hi - lo]
