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


# ---------------------------------------------------------------- read shards (C4 / C5 front end)
# One seed's results as they come back from a rank: the seed (bsw_seed_t), its read (rebased to the
# rank's first read) and chain, its region (bsw_alnreg_t) and the extended flag -- 17 int32.
REC_DTYPE = np.dtype([("seed", bsw.SEED_DTYPE), ("sr", "<i4"), ("sc", "<i4"), ("out", bsw.ALNREG_DTYPE),
                      ("ext", "<i4")])
REC_WORDS = REC_DTYPE.itemsize // 4
assert REC_DTYPE.itemsize == 68


def read_cut(n: int, world: int) -> np.ndarray:
    """contiguous read ranges of equal count (the C4 reads are all 150 bp: equal work per read)"""
    return np.array([n * k // world for k in range(world + 1)], dtype=np.int64)


def read_layout(n_k: int, nbytes: int) -> tuple:
    """byte offsets (reads, off int64, lens int32) inside one read-shard buffer, and its size"""
    o_off = (nbytes + 63) & ~63
    o_len = o_off + 8 * n_k
    return 0, o_off, o_len, o_len + 4 * n_k


def pack_reads(reads: np.ndarray, off: np.ndarray, lens: np.ndarray, cut):
    """[world, S] uint8: per range [read bytes | off (rebased) int64 | lens int32], padded to the
    largest; plus meta [world, 2] = (reads, read bytes)."""
    meta = []
    for k in range(len(cut) - 1):
        lo, hi = int(cut[k]), int(cut[k + 1])
        b0 = int(off[lo]) if hi > lo else 0
        b1 = int(off[hi - 1] + lens[hi - 1]) if hi > lo else 0
        meta.append((hi - lo, b1 - b0))
    meta = np.array(meta, dtype=np.int64).reshape(-1, 2)
    S = max([read_layout(int(n_k), int(nb))[3] for n_k, nb in meta] + [64])
    S = (S + 63) & ~63
    bufs = np.zeros((len(meta), S), dtype=np.uint8)
    for k in range(len(meta)):
        lo, hi = int(cut[k]), int(cut[k + 1])
        n_k, nb = int(meta[k, 0]), int(meta[k, 1])
        _, o_off, o_len, _ = read_layout(n_k, nb)
        if n_k == 0:
            continue
        b0 = int(off[lo])
        bufs[k, :nb] = reads[b0:b0 + nb]
        bufs[k, o_off:o_off + 8 * n_k] = (off[lo:hi].astype(np.int64) - b0).view(np.uint8)
        bufs[k, o_len:o_len + 4 * n_k] = lens[lo:hi].astype(np.int32).view(np.uint8)
    return bufs, meta


def unpack_reads(buf: np.ndarray, meta_row):
    """numpy views (reads, off, lens) into one read-shard buffer"""
    n_k, nb = int(meta_row[0]), int(meta_row[1])
    _, o_off, o_len, _ = read_layout(n_k, nb)
    return buf[:nb], buf[o_off:o_off + 8 * n_k].view(np.int64), buf[o_len:o_len + 4 * n_k].view(np.int32)


def merge_records(recs, counts, cut) -> np.ndarray:
    """Gathered per-rank record blocks (rank order, the first counts[k] rows valid) -> one REC
    array for the whole batch, reads renumbered to batch indices."""
    parts = []
    for k, (r, c) in enumerate(zip(recs, counts)):
        a = np.ascontiguousarray(np.asarray(r)[:int(c)]).view(REC_DTYPE).reshape(-1).copy()
        a["sr"] += int(cut[k])
        parts.append(a)
    return np.concatenate(parts) if parts else np.zeros(0, REC_DTYPE)


class ReadScatter:
    """The C5 front end as BASELINE configs[4] words it: ONE set of PE reads held by rank 0 (on
    GPU 0 in bench.py), cut into contiguous read ranges, `dist.scatter`ed one shard buffer per rank
    over `group` (RCCL in bench.py, gloo on CPU in the tests); every rank runs seeding -> chaining
    -> mem_chain2aln on its shard against its own copy of the index (built before timing) through
    `score(recv, meta_row, rec)` which fills rec[:ns] (REC_WORDS int32 per seed) and returns ns;
    the (count, records) blocks are gathered back to rank 0.  size(cap) fixes the record capacity
    (collective max over ranks after a sizing pass)."""

    def __init__(self, rank, world, group, device, reads=None, off=None, lens=None, meta_group=None):
        import torch
        import torch.distributed as dist
        self.rank, self.world, self.group, self.device = rank, world, group, device
        self._torch, self._dist = torch, dist
        self.meta_group = meta_group
        meta_t = torch.zeros((world, 2), dtype=torch.int64)
        self.src = None
        self.cut = None
        if rank == 0:
            self.cut = read_cut(len(lens), world)
            bufs, meta = pack_reads(reads, off, lens, self.cut)
            meta_t.copy_(torch.from_numpy(meta))
            self.src = [torch.from_numpy(bufs[k]).to(device) for k in range(world)]
            del bufs
        if world > 1:
            dist.broadcast(meta_t, src=0, group=meta_group)
        self.meta = meta_t.numpy().copy()
        self.n_me = int(self.meta[rank, 0])
        self.S = max(read_layout(int(a), int(b))[3] for a, b in self.meta)
        self.S = (self.S + 63) & ~63
        self.recv = torch.zeros(self.S, dtype=torch.uint8, device=device)
        self.cnt = torch.zeros(1, dtype=torch.int64, device=device)
        self.rec = None
        self.ms = {"scatter": [], "front_end": [], "gather": []}

    def layout(self):
        """(reads, off, lens) byte offsets of this rank's shard inside recv"""
        return read_layout(self.n_me, int(self.meta[self.rank, 1]))[:3]

    def size(self, cap: int):
        """record capacity: the max of every rank's `cap` (collective)"""
        torch = self._torch
        t = torch.tensor([cap], dtype=torch.int64)
        if self.world > 1:
            self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX, group=self.meta_group)
        self.cap = max(1, int(t.item()))
        self.rec = torch.zeros((self.cap, REC_WORDS), dtype=torch.int32, device=self.device)
        self.g_rec = ([torch.zeros_like(self.rec) for _ in range(self.world)] if self.rank == 0 else None)
        self.g_cnt = ([torch.zeros_like(self.cnt) for _ in range(self.world)] if self.rank == 0 else None)

    def _sync(self):
        if self.recv.is_cuda:
            self._torch.cuda.synchronize(self.recv.device)

    def scatter(self):
        if self.group is not None:
            self._dist.scatter(self.recv, self.src if self.rank == 0 else None, src=0, group=self.group)
        else:
            self.recv.copy_(self.src[0])
        self._sync()

    def step(self, score):
        import time
        t0 = time.perf_counter()
        self.scatter()
        t1 = time.perf_counter()
        ns = score(self.recv, self.meta[self.rank], self.rec) if self.n_me > 0 else 0
        if ns > self.cap:
            raise RuntimeError(f"rank {self.rank}: {ns} seeds past the record capacity {self.cap}")
        self.cnt.fill_(ns)
        t2 = time.perf_counter()
        if self.group is not None:
            self._dist.gather(self.cnt, self.g_cnt, dst=0, group=self.group)
            self._dist.gather(self.rec, self.g_rec, dst=0, group=self.group)
        self._sync()
        t3 = time.perf_counter()
        for k, a, b in (("scatter", t0, t1), ("front_end", t1, t2), ("gather", t2, t3)):
            self.ms[k].append((b - a) * 1e3)
        return ns

    def merged(self) -> np.ndarray:
        """rank 0: the whole batch's records (REC_DTYPE), reads numbered over the batch"""
        if self.group is None:
            return merge_records([self.rec.cpu().numpy()], [int(self.cnt.item())], self.cut)
        return merge_records([x.cpu().numpy() for x in self.g_rec], [int(x.item()) for x in self.g_cnt], self.cut)


class BatchScatter:
    """One fixed SeqPair batch held by rank 0, scored by every rank: the strong-scaling leg of
    bench.py (BASELINE configs[4]'s "RCCL-over-xGMI batch scatter") and of tests/test_dist.py.

    Construction (collective, untimed): rank 0 cuts the batch by static band cells, packs one
    buffer per rank (pack_shards) and keeps them on `device` (GPU 0 in bench.py); the per-rank
    meta goes to every rank over `meta_group` (gloo).  step(score) (collective, timed by the
    caller): `dist.scatter` of the shard buffers over `group` (backend "nccl" = RCCL in bench.py,
    gloo on CPU in the tests), `score(recv, meta_row)` on the received buffer in place (the
    caller's engine: bsw_get_scores_device on pointers into it, or the SSE4.1 restatement on
    numpy views), the 6 output int32 per pair copied out of the scored records, `dist.gather` of
    those blocks back to rank 0.  With group=None (one rank) a copy stands in for the scatter.
    merged() on rank 0: the whole batch's records with the gathered outputs written in."""

    def __init__(self, rank, world, group, device, pairs=None, ref=None, qer=None, w=100, meta_group=None):
        import torch
        import torch.distributed as dist
        self.rank, self.world, self.group, self.device = rank, world, group, device
        self._torch, self._dist = torch, dist
        meta_t = torch.zeros((world, 3), dtype=torch.int64)
        self.src = None
        self.pairs = self.cut = None
        if rank == 0:
            self.pairs = pairs
            self.cut = bsw.split_by_cells(pairs, w, world)
            bufs, meta = pack_shards(pairs, ref, qer, self.cut)
            meta_t.copy_(torch.from_numpy(meta))
            self.src = [torch.from_numpy(bufs[k]).to(device) for k in range(world)]
            del bufs
        if world > 1:
            dist.broadcast(meta_t, src=0, group=meta_group)
        self.meta = meta_t.numpy().copy()
        self.S = buffer_bytes(self.meta)
        self.n_me = int(self.meta[rank, 0])
        self.nmax = max(1, int(self.meta[:, 0].max()))
        self.recv = torch.zeros(self.S, dtype=torch.uint8, device=device)
        self.out_me = torch.zeros((self.nmax, 6), dtype=torch.int32, device=device)
        self.gathered = ([torch.zeros((self.nmax, 6), dtype=torch.int32, device=device) for _ in range(world)]
                         if rank == 0 else None)
        self.ms = {"scatter": [], "score": [], "gather": []}

    def _sync(self):
        if self.recv.is_cuda:
            self._torch.cuda.synchronize(self.recv.device)

    def step(self, score):
        import time
        dist = self._dist
        t0 = time.perf_counter()
        if self.group is not None:
            dist.scatter(self.recv, self.src if self.rank == 0 else None, src=0, group=self.group)
        else:
            self.recv.copy_(self.src[0])
        self._sync()                    # the engine runs on its own stream: the shard must be in
        t1 = time.perf_counter()
        n = self.n_me
        if n > 0:
            score(self.recv, self.meta[self.rank])
            po = offsets(self.meta[self.rank])[0]
            self.out_me[:n] = self.recv[po:po + 56 * n].view(self._torch.int32).view(n, 14)[:, OUT_COLS]
        t2 = time.perf_counter()
        if self.group is not None:
            dist.gather(self.out_me, self.gathered, dst=0, group=self.group)
        self._sync()
        t3 = time.perf_counter()
        for k, a, b in (("scatter", t0, t1), ("score", t1, t2), ("gather", t2, t3)):
            self.ms[k].append((b - a) * 1e3)

    def merged(self) -> np.ndarray:
        """rank 0: a copy of the batch with every rank's gathered outputs written in"""
        outs = ([x.cpu().numpy() for x in self.gathered] if self.group is not None
                else [self.out_me.cpu().numpy()])
        res = self.pairs.copy()
        merge_outputs(res, outs, self.cut)
        return res
