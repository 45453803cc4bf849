"""Multi-rank runs of the HIP engine (the N > 1 path of bench.py) on the GPU box.

Two ranks (torchrun, one process per rank, gloo for the control plane) share the box's one
GPU under --rehearse: bench.py --scaling strong splits ONE batch by static band cells
(bsw_split_by_cells), each rank scores its range through the host-buffer C ABI, rank 0
gathers the records.  The gathered outputs must equal the CPU oracle on the whole batch,
and the split must tile the batch.  (the 8-GPU curve is the driver's.)"""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import bsw
import oracle
from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2])
def test_ranks_strong_split_equal_oracle(tmp_path, world):
    n = 120_000
    dump = str(tmp_path / "out.npy")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--scaling", "strong", "--total-pairs", str(n),
           "--steps", "1", "--warmup", "1", "--rehearse", "--dump", dump]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["scaling"] == "strong" and line["n_gpus"] == world and "rehearsal" in line
    cut = line["config"]["cut"]
    assert cut[0] == 0 and cut[-1] == n and len(cut) == world + 1
    got = np.load(dump)
    assert got.dtype == bsw.SEQPAIR_DTYPE and len(got) == n
    full, ref, qer = bsw.synth_batch(n)
    want = full.copy()
    oracle.get_scores(oracle.make_params(), want, ref, qer, 100, nthreads=16)
    for f in ("len1", "len2", "h0") + bsw.OUT_FIELDS:
        assert np.array_equal(got[f], want[f]), f


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["c4", "c4mem"])
def test_ranks_c4_pe_workload_equal_oracle(tmp_path, workload):
    """The C4 / C5 workload (paired-end reads; c4: ground-truth seed chains through
    mem_chain2aln, c4mem: the whole GPU front end -- SMEM seeding, chaining, mem_chain2aln)
    under a 2-rank torchrun rehearsal on the box's one GPU: every rank's shard of reads
    (its own pair_base / read seed) equals the oracle run on that shard."""
    world, reads = 2, 20_000
    dump = str(tmp_path / "c4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--workload", workload, "--reads", str(reads),
           "--ref-mb", "4", "--steps", "1", "--warmup", "1", "--rehearse", "--no-cpu", "--dump", dump]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == world
    import bench
    import hiprt  # noqa: F401
    ref = bsw.synth_reference(4_000_000, seed=7)
    P = oracle.make_params()
    for rank in range(world):
        z = np.load(f"{dump}.rank{rank}.npz")
        if workload == "c4":
            npairs = reads // 2
            rd, off, lens, seeds, sr, sc = bsw.synth_pe_seeds(ref, npairs, pair_base=rank * npairs)
            want, wext = oracle.chain2aln(P, bsw.ext_opt(), ref, rd, off, lens, seeds, sr, sc, nthreads=8)
        else:
            nb = ref > 3
            ref2 = ref.copy()
            ref2[nb] = np.random.default_rng(1).integers(0, 4, int(nb.sum()), dtype=np.uint8)
            rd, off, lens = bench.pe_reads(ref2, reads // 2, seed=42 + rank)
            f = oracle.FmiRef(ref2)
            mems, cnt = f.collect_intv(rd, off, lens, cap=256, nthreads=8)
            seeds, sr, sc = oracle.mem_chain(f.sa(), len(ref2), lens, mems, cnt)
            assert np.array_equal(z["sr"], sr) and np.array_equal(z["sc"], sc)
            assert np.array_equal(z["seeds"]["rbeg"], seeds["rbeg"])
            T = np.concatenate([ref2, 3 - ref2[::-1]]).astype(np.uint8)
            want, wext = oracle.chain2aln(P, bsw.ext_opt(l_pac=len(ref2)), T, rd, off, lens, seeds, sr, sc, nthreads=8)
        assert np.array_equal(z["ext"], wext), f"rank {rank}"
        for fld in bsw.ALNREG_DTYPE.names:
            assert np.array_equal(z["out"][fld], want[fld]), (rank, fld)


@pytest.mark.gpu
def test_rccl_transport_one_rank_equal_oracle(tmp_path):
    """bench.py --scaling strong --transport rccl with one rank: the batch packed in the 2-bit wire
    form (bsw_pack_batch, three pieces), resident on GPU 0 as torch tensors, scattered by a one-rank
    RCCL communicator, each piece scored in place through bsw_get_scores_packed_device on its own
    stream and thread, the outputs gathered back through the same torch tensors RCCL moves.  (RCCL itself needs one GPU per rank: the N > 1 scatter /
    gather logic is covered over gloo by tests/test_dist.py; the 8-GPU run is the driver's.)"""
    n = 150_000
    dump = str(tmp_path / "rccl.npy")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--scaling", "strong", "--transport", "rccl",
           "--total-pairs", str(n), "--rccl-chunks", "3", "--steps", "2", "--warmup", "1", "--dump", dump]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["scaling"] == "strong" and line["n_gpus"] == 1 and "RCCL" in line["config"]["workload"]
    # a one-rank RCCL communicator carried the scatter / gather (backend nccl = RCCL on ROCm)
    assert line["rccl"]["rccl_world_size"] == 1 and line["rccl"]["backend"] == "nccl"
    assert line["rccl"]["outputs_identical_to_single_gpu"] is True
    # the 2-bit wire form (bsw_pack_batch), three pieces per rank scattered / scored / gathered
    assert line["rccl"]["chunks"] == 3 and line["rccl"]["wire_bytes_per_pair"] < 150
    got = np.load(dump)
    full, ref, qer = bsw.synth_batch(n)
    want = full.copy()
    oracle.get_scores(oracle.make_params(), want, ref, qer, 100, nthreads=16)
    for f in ("idr", "idq", "len1", "len2", "h0") + bsw.OUT_FIELDS:
        assert np.array_equal(got[f], want[f]), f


@pytest.mark.gpu
def test_rccl_read_scatter_c4mem_one_rank_equal_oracle(tmp_path):
    """bench.py --workload c4mem --scaling strong --transport rccl with one rank (BASELINE
    configs[4] on the whole front end): the PE reads packed into their read-shard buffer on GPU 0,
    scattered by a one-rank RCCL communicator, SMEM seeding -> chaining -> mem_chain2aln on the
    received buffer in place, the per-seed records gathered by RCCL -- equal to the oracle pipeline
    on the same reads at 4 Mb, and to the same job run directly on GPU 0."""
    reads = 20_000
    dump = str(tmp_path / "c5.npy")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c4mem", "--scaling", "strong",
           "--transport", "rccl", "--reads", str(reads), "--ref-mb", "4", "--steps", "2", "--warmup", "1",
           "--dump", dump]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["scaling"] == "strong" and line["rccl"]["rccl_world_size"] == 1
    assert line["rccl"]["backend"] == "nccl" and line["outputs_identical_to_single_gpu"] is True
    import bench
    import shards
    got = np.load(dump)
    assert got.dtype == shards.REC_DTYPE
    ref = bench.mem_reference(4)
    rd, off, lens = bench.pe_reads(ref, reads // 2, seed=42)
    f = oracle.FmiRef(ref)
    mems, cnt = f.collect_intv(rd, off, lens, cap=256, nthreads=8)
    seeds, sr, sc = oracle.mem_chain(f.sa(), len(ref), lens, mems, cnt)
    T = np.concatenate([ref, 3 - ref[::-1]]).astype(np.uint8)
    want, wext = oracle.chain2aln(oracle.make_params(), bsw.ext_opt(l_pac=len(ref)), T, rd, off, lens, seeds, sr, sc,
                                  nthreads=8)
    assert len(got) == len(seeds) and line["seeds"] == len(seeds)
    assert np.array_equal(got["sr"], sr) and np.array_equal(got["sc"], sc)
    assert np.array_equal(got["seed"], seeds)
    assert np.array_equal(got["ext"], wext)
    for fld in bsw.ALNREG_DTYPE.names:
        assert np.array_equal(got["out"][fld], want[fld]), fld


@pytest.mark.gpu
def test_two_rank_rehearsal_line_has_headline_keys():
    """bench.py --gpus 2 under torchrun with both ranks on GPU 0 (--rehearse): the N > 1 line the
    driver's scaling run prints, with the batch-scatter leg over gloo (ranks sharing a GPU cannot
    form an RCCL communicator) -- value = that leg's strong-scaling throughput, the per-rank
    resident rate in weak_value, the gathered outputs identical to the batch scored on one GPU."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--rehearse", "--steps", "3", "--warmup", "1", "--pairs", "100000",
           "--rccl-pairs", "300000", "--c5-reads", "0", "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["headline"].startswith("rccl_strong")
    leg = line["rccl_strong"]
    assert leg["backend"] == "gloo" and "rehearsal" in leg and leg["rccl_world_size"] == 2
    assert leg["outputs_identical_to_single_gpu"] is True and leg["total_pairs"] == 300_000
    assert line["value"] > 0 and line["weak_value"] > 0 and line["weak"]["scaling"] == "weak"
    assert (line["steps"], line["warmup"]) == (3, 1) and "rehearsal" in line
