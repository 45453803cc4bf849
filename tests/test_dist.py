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


def _scatter_worker(rank, world, port, n, q):
    """bench.py --scaling strong --transport rccl, on CPU tensors over gloo: rank 0 packs the
    whole batch (shards.py), scatters one padded buffer per rank, every rank scores its shard in
    place (the SSE4.1 restatement stands in for the GPU here), the 6 outputs per pair are
    gathered back to rank 0."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    import shards
    meta_t = torch.zeros((world, 3), dtype=torch.int64)
    src = None
    if rank == 0:
        pairs, ref, qer = bsw.synth_batch(n)
        pairs["len2"][::97] = 0                       # empty queries / targets inside a shard
        pairs["len1"][5::89] = 0
        cut = bsw.split_by_cells(pairs, 100, world)
        bufs, meta = shards.pack_shards(pairs, ref, qer, cut)
        meta_t.copy_(torch.from_numpy(meta))
        src = [torch.from_numpy(bufs[k].copy()) for k in range(world)]
    dist.broadcast(meta_t, src=0)
    meta = meta_t.numpy()
    recv = torch.zeros(shards.buffer_bytes(meta), dtype=torch.uint8)
    dist.scatter(recv, src, src=0)
    p, r, qq = shards.unpack_shard(recv.numpy(), meta[rank])
    oracle.sse41_get_scores16(oracle.make_params(), p, r, qq, 100, 1)
    nmax = int(meta[:, 0].max())
    out = torch.zeros((nmax, 6), dtype=torch.int32)
    out[:len(p)] = torch.from_numpy(shards.outputs(p))
    gathered = [torch.zeros_like(out) for _ in range(world)] if rank == 0 else None
    dist.gather(out, gathered, dst=0)
    if rank == 0:
        res = pairs.copy()
        shards.merge_outputs(res, [x.numpy() for x in gathered], cut)
        want = pairs.copy()
        oracle.get_scores(oracle.make_params(), want, ref, qer, 100)
        q.put(all(np.array_equal(res[f], want[f]) for f in bsw.OUT_FIELDS) and
              all(np.array_equal(res[f], pairs[f]) for f in ("idr", "idq", "len1", "len2", "h0")))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_scatter_gather_shards_equal_single_process(world):
    n = 1500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok
