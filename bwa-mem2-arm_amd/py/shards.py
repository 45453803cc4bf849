"""Batch scatter / gather over ranks -- BASELINE configs[4]'s "batch scatter" of SeqPair batches.

One batch (SeqPair records + the two byte buffers they index, upstream's layout) is cut into
contiguous pair ranges of equal static band cells (bsw_split_by_cells), one per
rank, and each range into `chunks` contiguous pieces.  Every piece travels in the engine's 2-bit
wire form (bsw_pack_batch, include/bsw.h: 20-B input records, 2-bit codes of the piece's byte
extents, an exception word per non-ACGT byte -- ~133 B per C2 pair instead of 56 + 450), one
scatter per chunk index, so chunk k + 1 moves while chunk k is scored; the rank scores each
received piece in place (bsw_get_scores_packed_device: one unpack kernel, then the device
pipeline) and its 24 output bytes per pair come back by one gather per chunk.  numpy here:
bench.py moves the buffers as torch tensors between the GPUs (backend "nccl" = RCCL over xGMI),
tests/test_dist.py as CPU tensors over gloo (with unpack_packed standing in for the device).

(Round 4 moved whole 56-B records + 1 byte per base in one unchunked scatter: pack_shards /
unpack_shard below, kept for the byte-layout tests.)"""

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
        self.error = None
        self.ms = {"scatter": [], "front_end": [], "gather": []}

    def agree_ok(self) -> bool:
        """collective over meta_group: True when no rank's score() failed"""
        t = self._torch.tensor([0 if self.error is None else 1], dtype=self._torch.int64)
        if self.world > 1:
            self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX, group=self.meta_group)
        return int(t.item()) == 0

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
        """one timed step; a score() failure (or more seeds than the capacity) is held in
        self.error and this rank sends 0 records, so every rank still takes part in the gathers
        (agree_ok() afterwards tells all ranks)"""
        import time
        t0 = time.perf_counter()
        self.scatter()
        t1 = time.perf_counter()
        try:
            ns = score(self.recv, self.meta[self.rank], self.rec) if self.n_me > 0 else 0
            if ns > self.cap:
                raise RuntimeError(f"rank {self.rank}: {ns} seeds past the record capacity {self.cap}")
        except Exception as e:  # noqa: BLE001
            self.error = self.error or e
            ns = 0
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


def unpack_packed(buf: np.ndarray, desc_row):
    """numpy inverse of bsw_pack_batch (test stand-in for the device unpack): (pairs, ref, qer)
    with idr / idq indexing the unpacked extents, outputs zeroed"""
    d = bsw.Packed.from_row(desc_row)
    n = d.n
    rec = buf[d.rec_off:d.rec_off + 20 * n].view(np.int32).reshape(n, 5)
    pairs = np.zeros(n, dtype=bsw.SEQPAIR_DTYPE)
    for k, f in enumerate(("idr", "idq", "len1", "len2", "h0")):
        pairs[f] = rec[:, k]

    def codes(off, nb, exc):
        b = buf[off:off + (nb + 3) // 4]
        out = np.stack([(b >> (2 * k)) & 3 for k in range(4)], axis=1).reshape(-1)[:nb].astype(np.uint8)
        pos = (exc >> 2).astype(np.int64)
        out[pos] = (out[pos] & 3) | ((exc & 3) << 2).astype(np.uint8)
        return out

    exc = buf[d.exc_off:d.exc_off + 4 * (d.n_exc_ref + d.n_exc_qer)].view(np.uint32)
    ref = codes(d.ref_off, d.ref_bytes, exc[:d.n_exc_ref])
    qer = codes(d.qer_off, d.qer_bytes, exc[d.n_exc_ref:])
    return pairs, ref, qer


WIRE_EXTENT_MAX = 1 << 30          # bsw_pack_batch: extents below 2^30 bytes (30-bit exception positions)


def pieces_fit(pairs: np.ndarray, cut, chunks: int) -> bool:
    """every rank's `chunks` pieces (chunk_cut) have ref and qer extents below WIRE_EXTENT_MAX"""
    for r in range(len(cut) - 1):
        lo, hi = int(cut[r]), int(cut[r + 1])
        cc = chunk_cut(hi - lo, chunks)
        for c in range(chunks):
            p = pairs[lo + int(cc[c]):lo + int(cc[c + 1])]
            for idx, ln in (("idr", "len1"), ("idq", "len2")):
                m = p[ln] > 0
                if m.any() and int((p[idx][m].astype(np.int64) + p[ln][m]).max() - p[idx][m].min()) >= WIRE_EXTENT_MAX:
                    return False
    return True


def chunk_cut(n: int, chunks: int) -> np.ndarray:
    """contiguous pieces of one rank's range (equal pair counts)"""
    return np.array([n * k // chunks for k in range(chunks + 1)], dtype=np.int64)


def pack_chunks(pairs: np.ndarray, ref: np.ndarray, qer: np.ndarray, cut, chunks: int):
    """rank 0's packing (untimed): per rank r and chunk c the wire form of rank r's piece c.
    Returns (bufs[r][c] uint8 arrays, desc [world, chunks, 10] int64, size [chunks]: the padded
    buffer size of chunk index c, the max over ranks, a multiple of 256)."""
    world = len(cut) - 1
    bufs = [[None] * chunks for _ in range(world)]
    desc = np.zeros((world, chunks, len(bsw.Packed.FIELDS)), dtype=np.int64)
    for r in range(world):
        lo, hi = int(cut[r]), int(cut[r + 1])
        cc = chunk_cut(hi - lo, chunks)
        for c in range(chunks):
            b, d = bsw.pack_batch(np.ascontiguousarray(pairs[lo + cc[c]:lo + cc[c + 1]]), ref, qer)
            bufs[r][c] = b
            desc[r, c] = d.to_row()
    size = np.array([max(256, (max(len(bufs[r][c]) for r in range(world)) + 255) & ~255) for c in range(chunks)],
                    dtype=np.int64)
    return bufs, desc, size


class BatchScatter:
    """One fixed SeqPair batch held by rank 0, scored by every rank: the strong-scaling leg of
    bench.py (BASELINE configs[4]'s "RCCL-over-xGMI batch scatter") and of tests/test_dist.py.

    Construction (collective, untimed): rank 0 cuts the batch by static band cells, each rank's
    range into `chunks` pieces, and packs every piece in the wire form (pack_chunks), keeping the
    buffers on `device` (GPU 0 in bench.py); the descriptors go to every rank over `meta_group`
    (gloo).  step(score) (collective, timed by the caller):
      - every chunk's `dist.scatter` is issued at once (async, in chunk order, over `group`: backend
        "nccl" = RCCL in bench.py, gloo in the tests);
      - one thread per chunk waits for its scatter (on its own stream in bench.py, so the wait is
        a device-side dependency) and calls score(c, recv[c], desc_row, out[c]) -- the engine's
        bsw_get_scores_packed_device in bench.py, the numpy unpack + SSE4.1 restatement in the
        tests -- which writes the piece's 6 output int32 per pair into out[c]; pieces of
        different chunks therefore overlap on the device (no per-chunk drain);
      - gathers of out[c] to rank 0, one per chunk, issued in chunk order as pieces finish.
    With group=None (one rank) copies stand in for the collectives.  A score() failure is held
    (self.error) while the collectives go on symmetrically -- one rank must not leave the others
    blocked in a collective -- and agree_ok() reports it to every rank afterwards.
    merged() on rank 0: the whole batch's records with the gathered outputs written in."""

    def __init__(self, rank, world, group, device, pairs=None, ref=None, qer=None, w=100, meta_group=None,
                 chunks=4):
        import torch
        import torch.distributed as dist
        self.rank, self.world, self.group, self.device = rank, world, group, device
        self._torch, self._dist = torch, dist
        self.meta_group = meta_group
        self.src = None
        self.pairs = self.cut = None
        # chunk count: at least `chunks`, and enough that every piece's byte extents stay inside
        # the wire form's 2^30-byte bound -- checked on the pieces as they will be cut (by pair
        # count: a skewed or permuted range can hold a long extent in one piece) -- then packed, all
        # on rank 0 before anything is broadcast; a failure there broadcasts -1 so every rank
        # raises together instead of leaving the others blocked in the broadcast below
        ch = torch.tensor([max(1, chunks)], dtype=torch.int64)
        bufs = desc = size = None
        err = None
        if rank == 0:
            try:
                self.pairs = pairs
                self.cut = bsw.split_by_cells(pairs, w, world)
                c = int(ch[0])
                while not pieces_fit(pairs, self.cut, c):
                    if c >= len(pairs):
                        raise ValueError("a single pair's extent passes the wire form's 2^30-byte bound")
                    c = min(2 * c, len(pairs))
                ch[0] = c
                bufs, desc, size = pack_chunks(pairs, ref, qer, self.cut, c)
            except Exception as e:  # noqa: BLE001  (re-raised below, on every rank)
                err = e
                ch[0] = -1
        if world > 1:
            dist.broadcast(ch, src=0, group=meta_group)
        if int(ch.item()) < 0:
            raise RuntimeError(f"BatchScatter: rank 0 could not pack the batch: {err!r}")
        chunks = self.chunks = int(ch.item())
        nf = len(bsw.Packed.FIELDS)
        meta_t = torch.zeros((world, chunks, nf + 1), dtype=torch.int64)
        if rank == 0:
            meta_t[:, :, :nf] = torch.from_numpy(desc)
            meta_t[:, :, nf] = torch.from_numpy(np.broadcast_to(size, (world, chunks)).copy())
            self.src = []
            for c in range(chunks):
                row = []
                for r in range(world):
                    t = torch.zeros(int(size[c]), dtype=torch.uint8)
                    t[:len(bufs[r][c])] = torch.from_numpy(bufs[r][c])
                    row.append(t.to(device))
                self.src.append(row)
            del bufs
        if world > 1:
            dist.broadcast(meta_t, src=0, group=meta_group)
        meta = meta_t.numpy().copy()
        self.desc = meta[:, :, :nf]
        self.size = meta[0, :, nf]
        self.n_me = int(self.desc[rank, :, 0].sum())
        self.nmax = [max(1, int(self.desc[:, c, 0].max())) for c in range(chunks)]
        self.S = int(self.size.sum())                  # wire bytes per rank (padded)
        self.wire_bytes = int(self.desc[:, :, -1].sum())   # total packed bytes of the batch
        self.recv = [torch.zeros(int(self.size[c]), dtype=torch.uint8, device=device) for c in range(chunks)]
        self.out = [torch.zeros((self.nmax[c], 6), dtype=torch.int32, device=device) for c in range(chunks)]
        self.gathered = ([[torch.zeros((self.nmax[c], 6), dtype=torch.int32, device=device) for _ in range(world)]
                          for c in range(chunks)] if rank == 0 else None)
        # one stream per chunk (the scoring thread's current stream: its scatter's wait and the
        # engine call are ordered on it)
        self.streams = ([torch.cuda.Stream(device=device) for _ in range(chunks)] if device.type == "cuda"
                        else None)
        self.error = None
        self.ms = {"scatter_first": [], "score_all": [], "gather_last": []}

    def _sync(self):
        if self.recv[0].is_cuda:
            self._torch.cuda.synchronize(self.recv[0].device)

    def _score_chunk(self, c, work, score, done):
        import contextlib
        ctx = (self._torch.cuda.stream(self.streams[c]) if self.streams is not None
               else contextlib.nullcontext())
        try:
            with ctx:
                if work is not None:
                    work.wait()
                if self.desc[self.rank, c, 0] > 0:
                    score(c, self.recv[c], self.desc[self.rank, c], self.out[c])
        except Exception as e:  # noqa: BLE001  (held: the collectives must go on on every rank)
            self.error = self.error or e
        finally:
            done[c] = __import__("time").perf_counter()

    def step(self, score):
        import threading
        import time
        dist = self._dist
        t0 = time.perf_counter()
        if self.group is not None:
            works = [dist.scatter(self.recv[c], self.src[c] if self.rank == 0 else None, src=0, group=self.group,
                                  async_op=True) for c in range(self.chunks)]
        else:
            for c in range(self.chunks):
                self.recv[c].copy_(self.src[c][0])
            works = [None] * self.chunks
        done = [0.0] * self.chunks
        th = [threading.Thread(target=self._score_chunk, args=(c, works[c], score, done))
              for c in range(self.chunks)]
        for t in th:
            t.start()
        gw = []
        for c, t in enumerate(th):
            t.join()
            if self.group is not None:
                gw.append(dist.gather(self.out[c], self.gathered[c] if self.rank == 0 else None, dst=0,
                                      group=self.group, async_op=True))
        t2 = time.perf_counter()
        for g in gw:
            g.wait()
        self._sync()
        t3 = time.perf_counter()
        self.ms["scatter_first"].append((done[0] - t0) * 1e3)
        self.ms["score_all"].append((t2 - t0) * 1e3)
        self.ms["gather_last"].append((t3 - t2) * 1e3)

    def agree_ok(self) -> bool:
        """collective over meta_group: True when no rank's score() failed"""
        torch = self._torch
        t = torch.tensor([0 if self.error is None else 1], dtype=torch.int64)
        if self.world > 1:
            self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX, group=self.meta_group)
        return int(t.item()) == 0

    def outputs_of(self, c, r):
        """rank 0: the gathered [n, 6] outputs of rank r's chunk c (numpy)"""
        n = int(self.desc[r, c, 0])
        src = self.gathered[c][r] if self.group is not None else self.out[c]
        return src[:n].cpu().numpy()

    def merged(self) -> np.ndarray:
        """rank 0: a copy of the batch with every rank's gathered outputs written in"""
        res = self.pairs.copy()
        v = res.view(np.int32).reshape(-1, 14)
        for r in range(self.world):
            lo, hi = int(self.cut[r]), int(self.cut[r + 1])
            cc = chunk_cut(hi - lo, self.chunks)
            for c in range(self.chunks):
                a, b = lo + int(cc[c]), lo + int(cc[c + 1])
                if b > a:
                    v[a:b, OUT_COLS] = self.outputs_of(c, r)
        return res
