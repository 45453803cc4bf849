"""Multi-process sharding on CPU (gloo, world_size 2) -- the N > 1 path of bench.py.

Pairs are independent: each rank generates and scores its own contiguous
shard [rank*n, (rank+1)*n) of the global synthetic batch; no data-path collective exists.
These tests check that the shards tile the single-process batch exactly, that per-shard
results equal the single-process results, and that the max-over-ranks timing reduction
used by bench.py behaves."""

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bsw
import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q, engine):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    pairs, ref, qer = bsw.synth_batch(n, pair_base=rank * n)
    if engine == "hip":            # the product engine (every rank on the box's GPU)
        e = bsw.Engine()
        e.get_scores(pairs, ref, qer, 100)
        e.close()
    else:                          # CPU container: the SSE4.1 restatement stands in per rank
        oracle.sse41_get_scores16(oracle.make_params(), pairs, ref, qer, 100, 1)
    out = torch.from_numpy(pairs.view(np.int32).reshape(n, 14).copy())
    gathered = [torch.zeros_like(out) for _ in range(world)]
    dist.all_gather(gathered, out)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((np.concatenate([g.numpy() for g in gathered]), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("engine", ["sse41", pytest.param("hip", marks=pytest.mark.gpu)])
def test_two_rank_shards_equal_single_process(engine):
    n, world = 600, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q, engine)) for r in range(world)]
    for p in procs:
        p.start()
    got, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == float(world)
    full, ref, qer = bsw.synth_batch(n * world)
    oracle.get_scores(oracle.make_params(), full, ref, qer, 100)
    got = got.view(bsw.SEQPAIR_DTYPE).reshape(-1)
    assert np.array_equal(got["id"], full["id"])
    for f in ("len1", "len2", "h0") + bsw.OUT_FIELDS:
        assert np.array_equal(got[f], full[f]), f


def test_synth_shards_tile_global_batch():
    a, ra, qa = bsw.synth_batch(300, pair_base=0)
    b, rb, qb = bsw.synth_batch(300, pair_base=300)
    full, rf, qf = bsw.synth_batch(600)
    assert np.array_equal(np.concatenate([ra, rb]), rf)
    assert np.array_equal(np.concatenate([qa, qb]), qf)
    assert np.array_equal(np.concatenate([a["h0"], b["h0"]]), full["h0"])


def _scatter_worker(rank, world, port, n, q, chunks, fail_rank):
    """bench.py's strong-scaling RCCL leg (rccl_c2_leg / --transport rccl) on CPU tensors over
    gloo, through the same orchestration code (shards.BatchScatter): rank 0 cuts the batch by band
    cells and packs every rank's range in `chunks` pieces of the 2-bit wire form (bsw_pack_batch),
    every chunk is scattered (async, all at once), each rank scores its pieces in place on one
    thread per chunk (numpy unpack + the SSE4.1 restatement stand in for the GPU), the 6 outputs
    per pair are gathered back to rank 0 chunk by chunk and merged; two steps, so the buffers are
    reused as in the timed loop.  fail_rank >= 0: that rank's score raises on chunk 0 of the
    second step -- every rank must still finish the step's collectives and then agree the leg
    failed."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    import shards
    pairs = ref = qer = None
    if rank == 0:
        pairs, ref, qer = bsw.synth_batch(n)
        pairs["len2"][::97] = 0                       # empty queries / targets inside a shard
        pairs["len1"][5::89] = 0
        qer[11::503] = 4                              # N bases: exception words of the wire form
        ref[3::701] = 4
    bs = shards.BatchScatter(rank, world, dist.group.WORLD, torch.device("cpu"), pairs, ref, qer, w=100,
                             meta_group=dist.group.WORLD, chunks=chunks)
    calls = []

    def score(c, recv, row, out):
        calls.append(c)
        if rank == fail_rank and len(calls) > chunks and c == 0:
            raise RuntimeError("injected")
        p, r, qq = shards.unpack_packed(recv.numpy(), row)
        oracle.sse41_get_scores16(oracle.make_params(), p, r, qq, 100, 1)
        out[:len(p)] = torch.from_numpy(shards.outputs(p))

    for _ in range(2):
        bs.step(score)
    ok = bs.agree_ok()
    if rank == 0:
        if fail_rank >= 0:
            q.put(not ok)
        else:
            res = bs.merged()
            want = pairs.copy()
            oracle.get_scores(oracle.make_params(), want, ref, qer, 100)
            q.put(ok and
                  all(np.array_equal(res[f], want[f]) for f in bsw.OUT_FIELDS) and
                  all(np.array_equal(res[f], pairs[f]) for f in ("idr", "idq", "len1", "len2", "h0")) and
                  all(len(v) == 2 for v in bs.ms.values()) and
                  int(bs.desc[:, :, 0].sum()) == n and bs.wire_bytes < n * 150)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,chunks,fail_rank", [(2, 1, -1), (2, 4, -1), (3, 3, -1), (3, 2, 1)])
def test_scatter_gather_shards_equal_single_process(world, chunks, fail_rank):
    n = 1500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, n, q, chunks, fail_rank))
             for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok


def test_packed_wire_form_roundtrip():
    """bsw_pack_batch (host-only) and its numpy inverse: records rebased to the extents, codes
    (incl. N and other non-ACGT bytes as exception words) and outputs of the oracle identical"""
    import shards
    pairs, ref, qer = bsw.synth_batch(3000)
    qer[5::97] = 4
    ref[7::131] = 4
    ref[9::1009] = 7                                   # any code outside 0..3 survives
    pairs["len1"][::50] = 0
    for lo, hi in ((0, 3000), (17, 1234), (2999, 3000), (5, 5)):
        sub = np.ascontiguousarray(pairs[lo:hi])
        buf, d = bsw.pack_batch(sub, ref, qer)
        assert d.n == hi - lo and d.total_bytes % 256 == 0 and d.total_bytes <= len(buf)
        p, r, qq = shards.unpack_packed(buf, d.to_row())
        for i in range(len(sub)):
            a, b = sub[i], p[i]
            assert (a["len1"], a["len2"], a["h0"]) == (b["len1"], b["len2"], b["h0"])
            assert np.array_equal(ref[a["idr"]:a["idr"] + a["len1"]], r[b["idr"]:b["idr"] + b["len1"]])
            assert np.array_equal(qer[a["idq"]:a["idq"] + a["len2"]], qq[b["idq"]:b["idq"] + b["len2"]])
        if hi - lo > 1000:
            assert d.n_exc_ref > 0 and d.n_exc_qer > 0
            assert d.total_bytes < (hi - lo) * 160        # vs 56 + 450 bytes per pair unpacked
            # scored on codes 0..4 (the ABI's alphabet; the oracle's 5x5 matrix has no row 7)
            w1, w2 = sub.copy(), p.copy()
            oracle.get_scores(oracle.make_params(), w1, np.minimum(ref, 4), qer, 100)
            oracle.get_scores(oracle.make_params(), w2, np.minimum(r, 4), qq, 100)
            for f in bsw.OUT_FIELDS:
                assert np.array_equal(w1[f], w2[f])


def test_packed_wire_form_errors():
    pairs, ref, qer = bsw.synth_batch(10)
    bad = pairs.copy()
    bad["len1"][3] = -1
    with pytest.raises(bsw.BswError):
        bsw.pack_batch(bad, ref, qer)
    big = pairs[:2].copy()
    big["idr"][1] = (1 << 30)                           # extent past 2^30 bytes
    with pytest.raises(bsw.BswError):
        bsw.pack_batch(big, np.zeros((1 << 30) + 400, np.uint8), qer)


def _read_scatter_worker(rank, world, port, nreads, q):
    """bench.py --workload c4mem --scaling strong --transport rccl on CPU tensors over gloo,
    through the same orchestration (shards.ReadScatter): rank 0 holds every PE read, the read
    shards are scattered, every rank runs the front end on its shard against its own index (the
    oracle pipeline -- FmiRef.collect_intv -> mem_chain -> chain2aln -- stands in for the GPU),
    the per-seed records are gathered and merged on rank 0."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    import bench
    import shards
    ref = bsw.synth_reference(300_000, seed=7)
    ref[ref > 3] = 0
    reads = off = lens = None
    if rank == 0:
        reads, off, lens = bench.pe_reads(ref, nreads // 2, seed=42)
        lens = lens.copy()
        lens[3] = 0                                   # an empty read inside a shard
    rs = shards.ReadScatter(rank, world, dist.group.WORLD, torch.device("cpu"), reads, off, lens)
    P = oracle.make_params()
    f = oracle.FmiRef(ref)                            # every rank its own index
    T = np.concatenate([ref, 3 - ref[::-1]]).astype(np.uint8)
    opt = bsw.ext_opt(l_pac=len(ref))

    def front_end(rd, of, ln):
        mems, cnt = f.collect_intv(rd, of, ln, cap=256, nthreads=1)
        seeds, sr, sc = oracle.mem_chain(f.sa(), len(ref), ln, mems, cnt)
        out, ext = oracle.chain2aln(P, opt, T, rd, of, ln, seeds, sr, sc, nthreads=1)
        return seeds, sr, sc, out, ext

    def score(recv, row, rec):
        seeds, sr, sc, out, ext = front_end(*shards.unpack_reads(recv.numpy(), row))
        ns = len(seeds)
        if rec is not None:
            r = rec.numpy()[:ns].view(shards.REC_DTYPE).reshape(-1)
            r["seed"], r["sr"], r["sc"], r["out"], r["ext"] = seeds, sr, sc, out, ext
        return ns

    rs.scatter()
    rs.size(score(rs.recv, rs.meta[rank], None) + 16)
    for _ in range(2):
        rs.step(score)
    if rank == 0:
        got = rs.merged()
        seeds, sr, sc, out, ext = front_end(reads, off, lens)
        q.put(bool(len(got) == len(seeds) and np.array_equal(got["seed"], seeds) and np.array_equal(got["sr"], sr)
                   and np.array_equal(got["sc"], sc) and np.array_equal(got["out"], out)
                   and np.array_equal(got["ext"], ext) and len(got) > nreads // 2
                   and int(rs.meta[:, 0].sum()) == nreads))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_read_scatter_gather_equal_single_process(world):
    nreads = 600
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_read_scatter_worker, args=(r, world, port, nreads, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok


def test_read_shard_pack_roundtrip():
    import shards
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 160, 101).astype(np.int32)
    off = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64) + 7
    reads = rng.integers(0, 5, int(off[-1] + lens[-1]) + 11).astype(np.uint8)
    for world in (1, 2, 3, 7):
        cut = shards.read_cut(len(lens), world)
        bufs, meta = shards.pack_reads(reads, off, lens, cut)
        assert int(meta[:, 0].sum()) == len(lens)
        for k in range(world):
            rd, of, ln = shards.unpack_reads(bufs[k], meta[k])
            lo, hi = int(cut[k]), int(cut[k + 1])
            assert np.array_equal(ln, lens[lo:hi])
            for i in range(hi - lo):
                assert np.array_equal(rd[of[i]:of[i] + ln[i]], reads[off[lo + i]:off[lo + i] + lens[lo + i]])


def _weak_line(world=2):
    return {"metric": "m", "value": 280.0, "unit": "u", "n_gpus": world, "steps": 20, "warmup": 5,
            "ms_per_step": 7.1, "scaling": "weak", "kernel_only_value": 290.0,
            "config": {"workload": "C2: 1000000 SeqPairs/GPU resident", "pairs_per_gpu": 1_000_000,
                       "parallelism": f"shard{world}"}}


def test_multi_gpu_line_headline_is_rccl_leg():
    """bench.py's N > 1 line: the RCCL batch-scatter leg's throughput is the value (strong scaling),
    the per-rank resident rate moves to weak_value / weak, the leg's details stay in rccl_strong"""
    import argparse
    import bench
    args = argparse.Namespace(w=100)
    leg = {"value": 850.0, "unit": "u", "scaling": "strong", "ms_per_step": 7.06, "steps": 20, "warmup": 5,
           "total_pairs": 6_000_000, "rccl_world_size": 8, "backend": "nccl",
           "outputs_identical_to_single_gpu": True}
    out = bench.multi_gpu_line(_weak_line(8), dict(leg), args, 8)
    assert out["value"] == 850.0 and out["scaling"] == "strong" and out["ms_per_step"] == 7.06
    assert (out["steps"], out["warmup"]) == (20, 5)
    assert out["weak_value"] == 280.0 and out["weak"]["scaling"] == "weak" and out["weak"]["ms_per_step"] == 7.1
    assert out["rccl_strong"]["rccl_world_size"] == 8 and "value" not in out["rccl_strong"]
    assert "RCCL scatter" in out["config"]["workload"] and out["config"]["total_pairs"] == 6_000_000
    assert "pairs_per_gpu" not in out["config"] and out["headline"].startswith("rccl_strong")
    # no RCCL value (skipped / failed): the weak rate stays the value, with the reason
    for bad in ({"skipped": "2 ranks share 1 GPU(s)"}, {"error": "RuntimeError('x')"}, None):
        o = bench.multi_gpu_line(_weak_line(2), bad, args, 2)
        assert o["value"] == 280.0 and o["scaling"] == "weak" and o["weak_value"] == 280.0
        assert o["headline"].startswith("weak")
        assert (bad is None) or o["rccl_strong"] == bad


def test_c5_guard_budget_and_memory(monkeypatch):
    """The C5 sub-object's guard: skipped with a stated reason when twice its projected time passes
    what is left of --budget-s or a rank's free device memory is below the index + buffers"""
    import argparse
    import bench
    import hiprt
    args = argparse.Namespace(c5_ref_mb=3000, c5_reads=10_000_000, budget_s=10_000.0)
    need = bench.c5_device_bytes(args, 0)
    assert 140e9 < need < 200e9                          # ~49.5 B per base of a 3 Gb index + buffers
    monkeypatch.setattr(hiprt, "mem_get_info", lambda: (280 << 30, 288 << 30))
    why, info = bench.c5_guard(args, 0, 1)
    assert why is None and info["projected_s"] > 0
    monkeypatch.setattr(hiprt, "mem_get_info", lambda: (100 << 30, 288 << 30))
    why, _ = bench.c5_guard(args, 0, 1)
    assert why and "device memory" in why
    monkeypatch.setattr(hiprt, "mem_get_info", lambda: (280 << 30, 288 << 30))
    args.budget_s = 1.0
    why, info = bench.c5_guard(args, 0, 1)
    assert why and "budget" in why and info["budget_s"] == 1.0
