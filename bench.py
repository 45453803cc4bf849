#!/usr/bin/env python3
"""bench.py -- M seed-extensions/s of the MI355X banded-SW engine (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): per GPU a resident synthetic SeqPair batch of
1,000,000 pairs, 150 bp query / 300 bp ref window, band w = 100, int16 cells, bwa-mem
default scoring (-A1 -B4 -O6 -E1 -d100 -L5); generator bwa-mem2-arm_amd/csrc/bsw_synth.c
(splitmix64 seed 42; 2% subs, 0.2% indels, 10% unrelated queries, 0.1% N, h0 U[19,100]).

One step = one bsw_get_scores_device() call over the whole resident batch (plan + sort +
DP kernel + results written back into the SeqPair records in HBM).  Inputs are resident in
HBM before timing starts.

N GPUs (one process per GPU, torchrun; control plane = torch.distributed/gloo): the line's value
is the RCCL batch scatter of BASELINE configs[4] -- ONE batch of --rccl-pairs C2 pairs (6M:
SeqPair's int32 idr addresses ~7M windows of 300 bytes) resident on GPU 0 in the 2-bit wire form,
scattered to the ranks' GPUs over an nccl (= RCCL) group, scored in place, outputs gathered back
to GPU 0, all timed over exactly --steps steps (strong scaling; rccl_world_size and the check that
the gathered outputs equal the same batch scored on GPU 0 alone are in rccl_strong).  Every rank
scoring its own resident 1M pairs with no data movement is reported beside it as weak_value.
C5 on the whole front end (the PE read set scattered, seeding -> chaining -> extension on every
rank, records gathered) follows in `c5` when --budget-s and every rank's free HBM allow it.

Reported beside the metric:
  roofline     -- dominant kernel (pc_kernel<160> on C2), integer-VALU bound: algorithmic ops
                  = 14 int ops x 25,100 static band cells per pair per
                  launch / HIP-event-timed launch duration, vs the gfx950 packed-int16 VALU
                  peak; traffic = HBM bytes per launch from the rocprofv3 PMC passes of THIS
                  workload (profiles/pmc_latest.json keyed by roofline.pmc_key), else null.
  cpu_baseline -- oracle/bsw_sse41.c (restated upstream SSE4.1 getScores16 design, "port")
                  on a bounded sample of the same batch; best of {affinity set, cgroup quota,
                  16} threads (model, core count and quota recorded), rank 0, N = 1 only.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time

T_START = time.perf_counter()
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))

import numpy as np  # noqa: E402

import hiprt  # noqa: E402  (loads the HIP runtime before anything imports torch)
import bsw  # noqa: E402

METRIC = "M seed-extensions/sec (150 bp, band=100) at 1/2/4/8 MI355X vs CPU"
UNIT = "M seed-extensions/s"
STATIC_CELLS_C2 = 25_100          # band cells per pair at 150/300, w=100
OPS_PER_CELL = 14                 # algorithmic int ops per cell
# gfx950 integer VALU peak, packed int16: 256 CU x 4 SIMD x 32 lanes x 2 (v_pk) x 2.4 GHz
VALU_PEAK_TOPS = 256 * 4 * 32 * 2 * 2.4e9 / 1e12


def static_band_cells(qlen: int, tlen: int, w: int, maxsc=1, end_bonus=5, o=6, e=1) -> int:
    wl = min(w, max((qlen * maxsc + end_bonus - o + e) // e, 1))
    return sum(max(0, min(qlen, i + wl + 1) - max(0, i - wl)) for i in range(tlen))


def wave_cols(qlen: int, w: int, maxsc=1, end_bonus=5, o=6, e=1) -> int:
    """columns per lane of the wave kernel for this shape (bsw_host.cpp wv_class)"""
    wl = min(w, max((qlen * maxsc + end_bonus - o + e) // e, 1))
    return next(c for c in (4, 8, 16) if 2 * wl + c + 2 <= 64 * c)


def dist_init():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    return rank, local, world


def allreduce_max(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(world: int):
    hiprt.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def workload_key(args) -> str:
    """The PMC lookup key of this run's workload: profiles/pmc_latest.json holds per workload key the
    kernels of the rocprofv3 PMC passes (tools/profile.sh) that ran exactly this workload
    (tools/pmc_summary.py reads the key from the profiled run's own JSON line, roofline.pmc_key)"""
    w = args.workload
    if w == "c2":
        return (f"c2:n{args.pairs}:q{args.qlen}:t{args.tlen}:w{args.w}:cb{args.cell_bits}:k8{args.kernel8}:"
                f"h{args.h0_hi}")
    if w in ("mate", "global"):
        return f"{w}:n{args.jobs}:ref{args.ref_mb}"
    if w == "smem":
        return f"smem:n{args.reads}:ref{args.smem_ref_mb}{':blocks' if args.fmi_blocks_only else ''}"
    if w == "c1":
        return "c1"
    pipe = f":p{args.pipeline}" if w == "c4mem" and getattr(args, "pipeline", 1) > 1 else ""
    return f"{w}:n{args.reads}:ref{args.ref_mb}:w{args.w}{':blocks' if args.fmi_blocks_only else ''}{pipe}"


def traffic_for(args, kernel: str, prefix: bool = False) -> dict:
    """HBM traffic of `kernel` (prefix: the longest-running kernel whose short name starts with it) per
    launch, from the PMC passes of THIS workload (workload_key) in profiles/pmc_latest.json:
    {"traffic": bytes, "traffic_kernel", "traffic_source", "counter_GBps": bytes / the traced
    average launch time}; traffic None when no pass of this workload measured the kernel -- a line
    never carries another workload's bytes"""
    key = workload_key(args)
    none = {"traffic": None, "traffic_source": f"no PMC pass of workload {key} in profiles/pmc_latest.json"}
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_latest.json")) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return none
    ent = d.get(key)
    if not isinstance(ent, dict):
        return none
    ks = ent.get("kernels", {})
    c = [(v.get("total_ns", 0), k, v) for k, v in ks.items()
         if (k.startswith(kernel) if prefix else k == kernel) and v.get("hbm_bytes_per_launch") is not None]
    if not c:
        return none
    _, k, v = max(c, key=lambda x: x[0])
    b = v["hbm_bytes_per_launch"]
    return {"traffic": b, "traffic_kernel": k, "traffic_source": ent.get("source"),
            "counter_GBps": round(b / v["avg_ns"], 1) if v.get("avg_ns") else None}


def host_cpu_info() -> dict:
    """What the CPU baseline ran on: usable cores (sched affinity), nproc-style count, the
    lscpu model string and any cgroup CPU quota (the box's real share may be below nproc)."""
    info = {"affinity_cores": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count()}
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    info["physical_cores"] = physical_cores()
    return info


def physical_cores():
    """Physical cores of the node (lscpu: sockets x cores per socket; else distinct
    (package, core) pairs in sysfs), independent of this process's affinity set or cgroup."""
    import subprocess
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {ln.split(":", 1)[0].strip(): ln.split(":", 1)[1].strip() for ln in out.splitlines() if ":" in ln}
        return int(kv["Socket(s)"]) * int(kv["Core(s) per socket"])
    except Exception:  # noqa: BLE001
        pass
    try:
        seen = set()
        base = "/sys/devices/system/cpu"
        for d in os.listdir(base):
            if d.startswith("cpu") and d[3:].isdigit():
                t = os.path.join(base, d, "topology")
                seen.add((open(os.path.join(t, "physical_package_id")).read().strip(),
                          open(os.path.join(t, "core_id")).read().strip()))
        return len(seen) or None
    except OSError:
        return None


def cpu_leg_threads() -> int:
    """threads for a multi-thread CPU baseline leg: the cgroup CPU quota (the box's real share)
    if set, else the affinity set, at most 64"""
    h = host_cpu_info()
    q = h.get("cgroup_cpu_quota")
    n = int(math.ceil(q)) if q else h["affinity_cores"]
    return max(1, min(64, n))


def node_extrapolation(rate, threads):
    phys = physical_cores()
    if not phys:
        return None
    return {"value": round(rate / threads * phys, 4), "physical_cores": phys,
            "note": "EXTRAPOLATED, not measured: the measured rate per thread x the node's physical cores (lscpu)"}


def _timed(fn, reps):
    """median wall time of `reps` runs after one warm-up"""
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts)


def cpu_baseline(pairs, ref, qer, w, gpu_pairs, cores):
    """oracle/bsw_sse41.c (the reference's SSE4.1 getScores16 design restated) on a bounded
    sample of the same batch, median of 5 after a warm-up (the reference's own script
    takes 3).  Thread counts tried: the reference's own sweep 1 / 2 / 4 / 8 / 16
    (benchmark_threading.sh:96-119) and the cgroup CPU
    quota (the box's real CPU share, which can be far below the affinity set; the affinity set
    itself only when no quota caps it -- oversubscribing the quota measures nothing); `value` is
    the BEST of them with `cores` = the count that gave it, the sweep beside it, plus the 1-thread
    SSE4.1 and scalar ksw_extend2 rates (BASELINE.md / north_star: core count stated)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # CPU baseline leg only (test infrastructure)
    P = oracle.make_params()
    host = host_cpu_info()
    quota = host.get("cgroup_cpu_quota")
    cap = min(cores, int(math.ceil(quota))) if quota else cores
    counts = sorted({c for c in (1, 2, 4, 8, 16) if c <= cap} | {cap})
    rates = {}
    best = None
    for c in counts:
        # ~12.5K pairs per thread (>= 0.1 s per run at ~0.1 M pairs/s/thread), at most the batch
        S = min(len(pairs), max(50_000, 12_500 * c))
        out = pairs[:S].copy()
        r = S / _timed(lambda: oracle.sse41_get_scores16(P, out, ref, qer, w, c), 5) / 1e6
        rates[c] = r
        if best is None or r > best[1]:
            best = (c, r, S, out)
    bc, bval, S, out = best
    S1 = min(len(pairs), 20_000)
    a = pairs[:S1].copy()
    t = time.perf_counter()
    oracle.sse41_get_scores16(P, a, ref, qer, w, 1)
    sse_1t = S1 / (time.perf_counter() - t) / 1e6
    S2 = min(len(pairs), 10_000)
    a = pairs[:S2].copy()
    t = time.perf_counter()
    oracle.get_scores(P, a, ref, qer, w, 1)
    scalar_1t = S2 / (time.perf_counter() - t) / 1e6
    agree = all(np.array_equal(out[f], gpu_pairs[:S][f]) for f in bsw.OUT_FIELDS)
    wider = wider_isa_legs(oracle, P, pairs, ref, qer, w, gpu_pairs, bc, S)
    cells = oracle.band_cells(P, pairs[:S2], ref, qer, w) / S2     # actual (narrowed) band cells per pair
    per_core = bval / bc
    phys = host.get("physical_cores")
    return {
        "value": round(bval, 4), "unit": UNIT, "cores": bc, "kind": "port",
        "per_core_rate": round(per_core, 5),
        "node_extrapolated": ({"value": round(per_core * phys, 3), "physical_cores": phys,
                               "note": "EXTRAPOLATED, not measured: per_core_rate (the best measured "
                                       "multi-thread rate / its threads) x the node's physical cores "
                                       "(lscpu); this box's cgroup gives the run fewer CPUs"}
                              if phys else None),
        "sample": f"first {S} pairs of the rank-0 C2 batch; oracle/bsw_sse41.c (SSE4.1, 8 x int16 "
                  f"lanes, restated upstream getScores16 design, not the upstream binary), {bc} threads "
                  f"(best of {counts} threads: the reference's 1/2/4/8/16 sweep and the cgroup quota "
                  f"{quota}; affinity set {cores}), median of 5 after 1 warm-up each",
        "host": host,
        "sse41_by_threads": {str(c): round(r, 4) for c, r in sorted(rates.items())},
        "sse41_1thread": round(sse_1t, 4), "scalar_ksw_extend2_1thread": round(scalar_1t, 4),
        "outputs_identical_to_gpu": bool(agree),
        "wider_isa_context": wider,
        "actual_cells_per_pair": round(cells, 1),
    }


def wider_isa_legs(oracle, P, pairs, ref, qer, w, gpu_pairs, threads, S):
    """Context beside the SSE4.1 baseline (upstream would dispatch its AVX-512BW
    kernels on an x86 host with them): the same batch restatement at 16 (AVX2) and 32
    (AVX-512BW) int16 lanes, oracle/bsw_avx512.c, at the thread count that gave the SSE4.1
    `value` and at 1 thread, on the same sample.  Not `value` -- north_star names SSE4.1."""
    legs = {}
    for isa in ("avx2", "avx512bw"):
        if not oracle.simd_supported(isa):
            legs[isa] = None
            continue
        out = pairs[:S].copy()
        r = S / _timed(lambda: oracle.simd_get_scores16(isa, P, out, ref, qer, w, threads), 5) / 1e6
        S1 = min(len(pairs), 20_000)
        a = pairs[:S1].copy()
        r1 = S1 / _timed(lambda: oracle.simd_get_scores16(isa, P, a, ref, qer, w, 1), 1) / 1e6
        legs[isa] = {"value": round(r, 4), "threads": threads, "1thread": round(r1, 4),
                     "outputs_identical_to_gpu": bool(all(np.array_equal(out[f], gpu_pairs[:S][f])
                                                          for f in bsw.OUT_FIELDS))}
    return legs


def coalesce_opt(eng):
    return getattr(eng, "coalesce_setting", 8192)


def host_path_rates(eng, pairs, ref, qer, w, cell_bits, want, curve_sizes=(1_000, 10_000, 100_000)):
    """The drop-in path: bsw_get_scores on HOST buffers (pageable numpy memory, as upstream's
    getScores16 caller hands them over), PCIe both ways included.  Whole batch (median of 3
    after a warm-up) and the per-call curve at upstream-like batch sizes (kt_for workers issue
    thousands of pairs per call): 1 calling thread, and 8 concurrent callers (each call takes
    its own slot/stream, ctypes releases the GIL).  Whole batch: median of 5 after a warm-up."""
    import threading
    n = len(pairs)
    buf = pairs.copy()
    ts = []
    eng.get_scores(buf, ref, qer, w, cell_bits)
    for _ in range(5):
        t = time.perf_counter()
        eng.get_scores(buf, ref, qer, w, cell_bits)
        ts.append(time.perf_counter() - t)
    t_all = statistics.median(ts)
    st = eng.last_stats()
    same = all(np.array_equal(buf[f], want[f]) for f in bsw.OUT_FIELDS)
    curve = []
    for m in curve_sizes:
        if m > n // 8:
            continue
        calls = max(20, min(200, int(2e6 // m)))
        lat = []
        for c in range(calls + 3):
            a = (c * m) % (n - m + 1)
            v = buf[a:a + m]
            t = time.perf_counter()
            eng.get_scores(v, ref, qer, w, cell_bits)
            lat.append(time.perf_counter() - t)
        lat = lat[3:]
        # 8 concurrent callers (ctypes releases the GIL), each over its own slice, calls back to
        # back for 0.5 s after every caller's untimed warm-up calls
        nthr, run_s = 8, 0.5
        slice_ = n // nthr
        go = threading.Barrier(nthr + 1)
        done = [0] * nthr

        def worker(k):
            for c in range(2):
                a = k * slice_ + (c * m) % (slice_ - m + 1)
                eng.get_scores(buf[a:a + m], ref, qer, w, cell_bits)
            go.wait()
            t0 = time.perf_counter()
            c = 0
            while time.perf_counter() - t0 < run_s:
                a = k * slice_ + ((c + 2) * m) % (slice_ - m + 1)
                eng.get_scores(buf[a:a + m], ref, qer, w, cell_bits)
                done[k] += m
                c += 1
        th = [threading.Thread(target=worker, args=(k,)) for k in range(nthr)]
        for x in th:
            x.start()
        go.wait()
        t = time.perf_counter()
        for x in th:
            x.join()
        dt8 = time.perf_counter() - t
        curve.append({"pairs_per_call": m, "latency_ms_median": round(statistics.median(lat) * 1e3, 3),
                      "M_pairs_per_s_1_caller": round(m / statistics.median(lat) / 1e6, 3),
                      "M_pairs_per_s_8_callers": round(sum(done) / dt8 / 1e6, 3),
                      "seconds_8_callers": round(dt8, 3)})
    return {"value": round(n / t_all / 1e6, 3), "ms": round(t_all * 1e3, 3),
            "coalesce_max_pairs": coalesce_opt(eng),
            "ms_all_calls": [round(x * 1e3, 2) for x in ts],
            "last_call": {"host_ms": round(st.host_ms, 3), "stage_ms": round(st.stage_ms, 3),
                          "dp_kernel_ms": round(st.kernel_ms, 3), "launches": st.n_launches},
            "outputs_identical_to_resident": bool(same), "per_call_curve": curve}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    # default C2 run: 100 x ~7 ms, a timed region of ~0.7 s (long enough for an outside
    # utilisation sampler); the other workloads: 10 steps, 2 warm-up
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--pairs", type=int, default=1_000_000, help="pairs per GPU")
    ap.add_argument("--w", type=int, default=100)
    ap.add_argument("--cell-bits", type=int, default=16, choices=(8, 16))
    ap.add_argument("--h0-hi", type=int, default=100, help="h0 upper bound (C3 uses 105)")
    ap.add_argument("--kernel8", type=int, default=1, choices=(0, 1, 2),
                    help="BSW_OPT_KERNEL8 for the 8-bit-regime pairs: 1 packed-column kernel (default), 2 the same "
                         "with byte-wide H/E planes (8-bit cells, 3 waves/SIMD at QMAX 160), 0 int16 lane kernel")
    ap.add_argument("--qlen", type=int, default=150, help="query length (C2: 150; long reads: 250 / 500 / 1000)")
    ap.add_argument("--tlen", type=int, default=300, help="target window length (C2: 300)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-host-path", action="store_true", help="skip the host-buffer (drop-in ABI) rates")
    ap.add_argument("--workload", default="c2", choices=("c2", "c1", "c4mem", "c4", "c4seed", "mate", "global", "smem"),
                    help="c2 (default): resident SeqPair batch; c1: the reference's own 10K exact SE reads vs "
                         "its 1 Mb reference through GPU seeding -> chaining -> mem_chain2aln; c4mem: the same "
                         "front end on --reads PE reads vs a --ref-mb reference; "
                         "c4: paired-end reads with several seeds / chains each through mem_chain2aln "
                         "(bsw_chain2aln_device); c4seed: one seed per read through the extension pipeline; "
                         "mate: resident mate-rescue batch (ksw_align2 jobs, SURVEY.md §8(f) row 2); "
                         "global: resident ksw_global2 + CIGAR batch (SURVEY.md §8(f) row 4)")
    ap.add_argument("--jobs", type=int, default=1_000_000, help="mate: jobs per GPU")
    ap.add_argument("--reads", type=int, default=1_000_000, help="c4: reads per GPU per step")
    ap.add_argument("--ref-mb", type=int, default=64, help="c4: random reference size (Mb)")
    ap.add_argument("--smem-ref-mb", type=int, default=16, help="smem: reference size (Mb) of the FM-index")
    ap.add_argument("--fmi-blocks-only", action="store_true",
                    help="smem / c1 / c4mem: index without the text-mode data (BSW_FMI_NO_TEXT; A/B)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="c4mem: split the step's reads into this many batches and run batch k's mem_chain2aln "
                         "(VALU-bound extension kernels, the engine's streams) on a second host thread while "
                         "batch k + 1 is seeded and chained (latency-bound SMEM walk, the index's stream); 1 = "
                         "the three stages back to back over every read")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                    help="weak (default): every rank scores its own resident 1M-pair shard; strong: one "
                         "fixed batch of --total-pairs split over the ranks by band cells, host buffers "
                         "in, PCIe both ways inside the timed region (C5)")
    ap.add_argument("--total-pairs", type=int, default=10_000_000, help="strong: pairs in the whole batch")
    ap.add_argument("--rccl-chunks", type=int, default=None,
                    help="RCCL C2 leg: pieces per rank (chunk k + 1 scatters while chunk k is scored).  Default 2 "
                         "at one rank (no scatter to hide: 2 pieces 0.946-0.968 of the single-GPU time, 4 pieces "
                         "0.941-0.949, profiles/r06/rccl_leg_trace.txt), 4 at N > 1 (the first piece's scatter "
                         "over xGMI is exposed: smaller pieces start each rank's DP sooner)")
    ap.add_argument("--rccl-pairs", type=int, default=6_000_000,
                    help="default C2 line at N > 1: pairs of the strong-scaling RCCL leg whose throughput is the "
                         "line's value (one batch on GPU 0, RCCL scatter -> score -> RCCL gather; the per-rank "
                         "resident rate is weak_value); 0 = off (the weak rate is the value)")
    ap.add_argument("--c5-reads", type=int, default=10_000_000,
                    help="default C2 line at N > 1: PE reads of the C5 sub-object (BASELINE configs[4]: the read "
                         "set resident on GPU 0, RCCL read scatter, the whole GPU front end on every rank, records "
                         "gathered); 0 = off")
    ap.add_argument("--c5-ref-mb", type=int, default=3000, help="C5 sub-object: reference size (Mb)")
    ap.add_argument("--budget-s", type=float, default=600.0,
                    help="N > 1: wall-clock budget of the whole run (the driver's timeout is not published); "
                         "the C5 sub-object runs only when twice its projected time fits what is left")
    ap.add_argument("--transport", default="host", choices=("host", "rccl"),
                    help="strong: host (default) -- every rank holds its range in host memory and the call "
                         "stages it over its own PCIe link; rccl -- the whole batch resident on GPU 0, scattered "
                         "to the ranks' GPUs and the outputs gathered back with RCCL over xGMI "
                         "(torch.distributed backend nccl), BASELINE configs[4]'s batch scatter")
    ap.add_argument("--rehearse", action="store_true",
                    help="allow more ranks than visible GPUs (ranks share GPUs; rehearsal only)")
    ap.add_argument("--dump", default="", help="strong: rank 0 writes the gathered outputs here (.npy); c4 / "
                                               "c4mem: every rank writes <dump>.rank<r>.npz")
    args = ap.parse_args()
    c2_default = args.workload == "c2" and args.scaling == "weak"
    if args.steps is None:
        args.steps = 100 if c2_default else 10
    if args.warmup is None:
        args.warmup = 5 if c2_default else 2

    rank, local, world = dist_init()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.rccl_chunks is None:
        args.rccl_chunks = 2 if world == 1 else 4
    ndev = hiprt.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no HIP device visible")
    if local >= ndev and not args.rehearse:
        raise SystemExit(f"bench.py: rank {rank} has LOCAL_RANK {local} but only {ndev} GPU(s) are visible; "
                         f"--rehearse lets ranks share GPUs (never a scaling measurement)")
    args.distinct_gpus = min(world, ndev)
    local = local % ndev              # --rehearse: more ranks than GPUs share them
    hiprt.set_device(local)
    if args.scaling == "strong":
        if args.transport == "rccl":
            if args.workload == "c4mem":
                return main_mem_strong_rccl(args, rank, local, world)
            return main_strong_rccl(args, rank, local, world)
        return main_strong(args, rank, local, world)
    if args.workload == "c1":          # BASELINE configs[0]: 10K exact 150 bp SE reads vs 1 Mb
        return main_mem(args, rank, local, world, c1=True)
    if args.workload == "c4mem":
        return main_mem(args, rank, local, world, c1=False)
    if args.workload == "c4":
        return main_c4pe(args, rank, local, world)
    if args.workload == "c4seed":
        return main_c4(args, rank, local, world)
    if args.workload == "mate":
        return main_mate(args, rank, local, world)
    if args.workload == "global":
        return main_global(args, rank, local, world)
    if args.workload == "smem":
        return main_smem(args, rank, local, world)

    cfg = bsw.synth_cfg(h0_hi=args.h0_hi, qlen=args.qlen, tlen=args.tlen)
    t0 = time.perf_counter()
    pairs, ref, qer = bsw.synth_batch(args.pairs, pair_base=rank * args.pairs, cfg=cfg)
    gen_s = time.perf_counter() - t0
    d_pairs = hiprt.DeviceBuffer.from_array(pairs)
    d_ref = hiprt.DeviceBuffer.from_array(ref)
    d_qer = hiprt.DeviceBuffer.from_array(qer)
    eng = bsw.Engine(device=local)
    if args.kernel8 != 1:
        eng.set_option("kernel8", args.kernel8)

    def step():
        eng.get_scores_device(d_pairs.ptr, d_ref.ptr, d_qer.ptr, args.pairs, args.w, args.cell_bits)

    for _ in range(args.warmup):
        step()
    kms = []
    barrier(world)
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
        kms.append(eng.last_stats().kernel_ms)
    barrier(world)
    dt = time.perf_counter() - t
    dt_max = allreduce_max(dt, world)
    st = eng.last_stats()

    res = np.empty_like(pairs)
    d_pairs.download(res)
    # N > 1: the HEADLINE is the RCCL batch scatter (BASELINE configs[4]): one batch resident on
    # GPU 0, scattered over the ranks by RCCL, scored, outputs gathered back -- timed over exactly
    # --steps steps after --warmup; the weak rate above (every rank its own resident 1M pairs, no
    # data movement) is reported beside it as weak_value.  C5 on the whole front end follows when
    # the run's wall-clock budget and every rank's free device memory allow it.  Each leg's ranks
    # agree over gloo before and after their RCCL phases, so a failing rank makes the leg report
    # an error on every rank instead of leaving the others blocked in a collective
    rccl = c5 = None
    budget = {}
    if world > 1:
        share = f"{world} ranks share {args.distinct_gpus} GPU(s) (--rehearse): RCCL needs one GPU per rank"
        def leg(fn, *a, **k):
            try:
                return fn(*a, **k)
            except Exception as e:  # noqa: BLE001  (symmetric failures: every rank lands here)
                return {"error": repr(e)[:400]}
        if args.rccl_pairs > 0:
            # ranks sharing a GPU (--rehearse) cannot form an RCCL communicator: the same leg then runs
            # with a gloo group over host-staged buffers (every key of the real line, labelled)
            rccl = leg(rccl_c2_leg, args, rank, local, world, args.rccl_pairs, steps=args.steps, warmup=args.warmup,
                       eng=eng, transport="nccl" if args.distinct_gpus >= world else "gloo")
        if args.c5_reads > 0:
            if args.distinct_gpus < world:
                c5 = {"skipped": share}
            else:
                why, budget = c5_guard(args, rank, world)
                c5 = {"skipped": why, "budget": budget} if why else \
                    leg(rccl_c5_leg, args, rank, local, world, args.c5_reads, args.c5_ref_mb, steps=5, warmup=1)
    if rank != 0:
        return
    total_pairs = args.pairs * world * args.steps
    value = total_pairs / dt_max / 1e6
    kms_mean = float(np.mean(kms))
    per_launch_pairs = args.pairs if st.n_launches == 1 else None
    cells = STATIC_CELLS_C2 if (cfg.qlen, cfg.tlen, args.w) == (150, 300, 100) else \
        static_band_cells(cfg.qlen, cfg.tlen, args.w)
    achieved = (args.pairs * cells * OPS_PER_CELL) / (kms_mean * 1e-3) / 1e12
    # the dominant launch: the packed-column kernel when the batch is in the 8-bit score
    # regime (C2: every pair; C3: most, the rest on the int16 lane kernel), else the lane
    # kernel; BSW_PK=1 selects the two-pairs-per-lane kernel for those pairs instead
    packed = 2 * st.n_packed > args.pairs
    wave = 2 * st.n_wave > args.pairs
    group = 2 * st.n_group > args.pairs              # small batches: the row-group kernel (device
    kname = ("gq_kernel<10>" if group else           #   calls run its 10-column form)
             ("pc_kernel<160,bytes>" if args.kernel8 == 2 else "pc_kernel<160>") if packed else (f"wv_kernel<{wave_cols(cfg.qlen, args.w)}>" if wave
                                              else "lane_kernel<160>"))
    roof = {
        "bound": "valu", "achieved": round(achieved, 3), "peak": round(VALU_PEAK_TOPS, 1),
        "unit": "TOP/s", "frac": round(achieved / VALU_PEAK_TOPS, 4),
        **traffic_for(args, kname), "pmc_key": workload_key(args),
        "kernel": kname, "launch_ms": round(kms_mean, 4),
        "cells_per_s": round(args.pairs * cells / (kms_mean * 1e-3) / 1e12, 4),
        "cells_unit": f"T band cells/s ({cells:,} static cells/pair)",
        "algorithmic": f"{OPS_PER_CELL} int ops x {cells} band cells x {args.pairs} pairs per launch",
        "pairs_per_launch": per_launch_pairs,
    }
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": UNIT, "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": ("u8 cells (byte H/E planes, int16 arithmetic)" if args.kernel8 == 2 and packed else
                                                   "int16" if args.cell_bits == 16 else "u8+int16"),
        "data": "synthetic (bsw_synth.c, seed 42)",
        "config": {"workload": f"{'C3' if args.cell_bits == 8 else 'C2' if cfg.qlen <= 160 else 'long reads'}: {args.pairs} SeqPairs/GPU resident in HBM, {cfg.qlen} bp query / "
                               f"{cfg.tlen} bp ref, band w={args.w}, cell_bits={args.cell_bits}, "
                               f"{'byte-plane kernel8=2, ' if args.kernel8 == 2 else ''}"
                               f"h0 U[{cfg.h0_lo},{cfg.h0_hi}]",
                   "pairs_per_gpu": args.pairs, "parallelism": f"shard{world} (independent pairs)",
                   "distinct_gpus": args.distinct_gpus,
                   "routing": {"n_packed": st.n_packed, "n_i16": st.n_i16, "n_u8": st.n_u8, "n_wide": st.n_wide,
                               "n_wave": st.n_wave, "n_group": st.n_group,
                               "int16_fallback_fraction": (round(st.n_i16 / max(1, st.n_i16 + st.n_u8), 4)
                                                           if args.cell_bits == 8 else None)}},
        "roofline": roof,
        "kernel_only_value": round(args.pairs * world / (kms_mean * 1e-3) / 1e6, 3),
    }
    if wave and world == 1:
        # the same resident batch on the int32 wide kernel (BSW_OPT_LONG 0): what long queries
        # ran on before the wave kernel
        e0 = bsw.Engine(device=local, long=0)
        e0.get_scores_device(d_pairs.ptr, d_ref.ptr, d_qer.ptr, args.pairs, args.w, args.cell_bits)
        t = time.perf_counter()
        e0.get_scores_device(d_pairs.ptr, d_ref.ptr, d_qer.ptr, args.pairs, args.w, args.cell_bits)
        wide_s = time.perf_counter() - t
        out["wide_kernel_comparison"] = {"M_pairs_per_s": round(args.pairs / wide_s / 1e6, 3),
                                         "dp_kernel_ms": round(e0.last_stats().kernel_ms, 3),
                                         "n_wide": e0.last_stats().n_wide}
        e0.close()
    if args.distinct_gpus < world:
        out["rehearsal"] = f"{world} ranks on {args.distinct_gpus} GPU(s): not a scaling measurement"
    if world > 1:
        out = multi_gpu_line(out, rccl, args, world)
    if c5 is not None:
        out["c5"] = dict(c5, workload=f"C5 (BASELINE configs[4]): {args.c5_reads} PE 150 bp reads vs a "
                                      f"{args.c5_ref_mb} Mb random reference, RCCL read scatter over {world} GPUs")
    if world == 1 and not args.no_host_path:
        hp = host_path_rates(eng, pairs, ref, qer, args.w, args.cell_bits, res)
        out["abi_inclusive_value"] = hp.pop("value")
        out["abi_inclusive"] = dict(hp, unit=UNIT, note="bsw_get_scores on pageable host buffers: staging "
                                    "(2-bit codes, 20-B input records) + H2D + plan/sort/DP + D2H of the outputs, "
                                    "chunked pipeline over four slots")
        eng.set_option("host_pack", 4)                 # the nibble staging beside it (same box, same batch)
        hp4 = host_path_rates(eng, pairs, ref, qer, args.w, args.cell_bits, res, curve_sizes=())
        eng.set_option("host_pack", 2)
        out["abi_inclusive"]["nibble_staging"] = {"value": hp4["value"], "ms": hp4["ms"],
                                                  "outputs_identical_to_resident": hp4["outputs_identical_to_resident"]}
        # the same curve from C++ kt_for-style threads through the C ABI (tools/percall_bench.cpp:
        # no Python between calls), with and without cross-call coalescing -- in a process of its own,
        # after this one has released its engine: the engine's slot streams each hold a hardware
        # queue, and with both processes' queues on the GPU the 8 x 10K point read 37 M/s instead of
        # the 41-42 the same binary measures alone (profiles/r06/percall_10k_quad_ab.txt)
        eng.close()
        for b in (d_pairs, d_ref, d_qer):
            b.free()
        import subprocess
        exe = os.path.join(ROOT, "bwa-mem2-arm_amd", "lib", "percall_bench")
        if os.path.exists(exe):
            try:
                r = subprocess.run([exe, "1000000", "8", "1000", "10000", "100000"], capture_output=True, text=True,
                                   timeout=120)
                if r.returncode == 0:
                    out["abi_inclusive"]["per_call_curve_cpp_callers"] = json.loads(r.stdout.strip().splitlines()[-1])
            except (subprocess.SubprocessError, ValueError, IndexError):
                pass
    if world == 1 and not args.no_cpu:
        cores = args.cpu_threads or len(os.sched_getaffinity(0))
        out["cpu_baseline"] = cpu_baseline(pairs, ref, qer, args.w, res, cores)
        out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 2)
        ne = out["cpu_baseline"].get("node_extrapolated")
        if ne:
            out["speedup_vs_cpu_node_extrapolated"] = round(value / ne["value"], 2)
        wl = [(k, v) for k, v in (out["cpu_baseline"].get("wider_isa_context") or {}).items() if v]
        if wl:
            isa, leg = max(wl, key=lambda kv: kv[1]["value"])
            out["speedup_vs_widest_isa"] = {"isa": isa, "vs_measured": round(value / leg["value"], 2)}
            phys = out["cpu_baseline"]["host"].get("physical_cores")
            if phys:
                out["speedup_vs_widest_isa"]["vs_node_extrapolated"] = round(
                    value / (leg["value"] / leg["threads"] * phys), 2)
        # achieved rate on the cells the literal loop really visits (10K-pair sample of the batch)
        acp = out["cpu_baseline"].pop("actual_cells_per_pair")
        roof["actual_cells_per_pair"] = acp
        roof["actual_cells_per_s"] = round(args.pairs * acp / (kms_mean * 1e-3) / 1e12, 4)
    out["synth_gen_s"] = round(gen_s, 2)
    print(json.dumps(out), flush=True)


def multi_gpu_line(out: dict, rccl, args, world: int) -> dict:
    """The N > 1 line: value = the RCCL batch-scatter leg's throughput (strong scaling: one batch of
    --rccl-pairs C2 pairs from GPU 0 over every rank, scatter + score + gather timed), with the
    per-rank resident rate kept as weak_value / weak.  When the RCCL leg did not produce a value
    (ranks sharing GPUs, --rccl-pairs 0, or a failure, reported in rccl_strong) the weak rate stays
    the value and `headline` says why."""
    weak = {k: out[k] for k in ("value", "ms_per_step", "steps", "warmup", "kernel_only_value")}
    weak["scaling"] = "weak"
    weak["workload"] = out["config"]["workload"]
    if rccl is None or "value" not in rccl:
        out["weak_value"] = out["value"]
        out["headline"] = ("weak: every rank's own resident batch (the RCCL batch-scatter leg did not run: "
                           f"{(rccl or {}).get('skipped') or (rccl or {}).get('error') or '--rccl-pairs 0'})")
        if rccl is not None:
            out["rccl_strong"] = rccl
        return out
    leg = dict(rccl)
    out["weak_value"] = weak.pop("value")
    out["weak"] = weak
    out["value"] = leg.pop("value")
    out["ms_per_step"] = leg.pop("ms_per_step")
    out["steps"], out["warmup"] = leg.pop("steps"), leg.pop("warmup")
    out["scaling"] = leg.pop("scaling")
    out["headline"] = "rccl_strong: one batch on GPU 0, RCCL scatter -> score -> RCCL gather (weak rate in weak_value)"
    out["config"] = dict(out["config"], workload=(
        f"C5 batch scatter (BASELINE configs[4]): one batch of {leg['total_pairs']} C2 pairs (150 bp query / 300 bp "
        f"ref, w={args.w}) resident on GPU 0 in the 2-bit wire form, split over {world} ranks by static band cells, "
        f"RCCL scatter -> bsw_get_scores_packed_device -> RCCL gather of the outputs, all inside the timed region"),
        total_pairs=leg["total_pairs"], parallelism=f"split{world} (bsw_split_by_cells; RCCL scatter + gather)")
    out["config"].pop("pairs_per_gpu", None)
    out["kernel_only_value"] = None                # a per-rank kernel rate: in weak
    out["rccl_strong"] = leg
    return out


# Wall-clock guard of the N > 1 line's secondary legs.  The driver runs `bench.py --gpus N` under a
# timeout it does not publish; --budget-s (default 600 s) is the assumed limit for the whole run,
# counted from the process start (T_START).  A leg starts only if the time left covers twice its
# projection.


def c5_projection_s(args, world: int) -> float:
    """Projected wall time of rccl_c5_leg (steps 5, warmup 1), from the round-6 one-rank 3 Gb run
    (profiles/r06/c5_one_rank_3gb.json): every rank generates the reference (~6 s per Gb) and builds
    its index on its GPU (~1 s per Gb incl. the two-strand text upload); rank 0 generates the reads
    (~1 s per M reads); sizing + warm-up + 5 steps over 1/world of the reads each (~25 ms per M reads
    per step on one GPU), then the one-GPU rerun of the whole set (3 x) and the record check."""
    gb = args.c5_ref_mb / 1000.0
    mr = args.c5_reads / 1e6
    return 7.0 * gb + 1.0 * mr + (7 * 0.025 * mr) / world + 4 * 0.025 * mr + 0.3 * mr + 10.0


def c5_device_bytes(args, rank: int) -> int:
    """Device bytes rccl_c5_leg needs on a rank: the wide FM-index (~47.5 B per reference base,
    profiles/r05: 142.6 GB at 3 Gb) + the two-strand text for extension (2 B per base) + the read
    shard and front-end buffers; rank 0 also holds the whole read set, the gathered records and a
    one-GPU front end over every read (~1.3 KB per read at 64 interval slots)"""
    bases = args.c5_ref_mb * 1_000_000
    reads = args.c5_reads
    per_read = 1300
    return int(49.5 * bases + per_read * reads * (2 if rank == 0 else 1) + (8 << 30))


def c5_guard(args, rank: int, world: int):
    """(reason to skip, budget dict) -- collective: every rank checks its free device memory, rank 0
    the time budget; the ranks agree over gloo, so all skip or all run"""
    free, total = hiprt.mem_get_info()
    need = c5_device_bytes(args, rank)
    left = args.budget_s - (time.perf_counter() - T_START)
    proj = c5_projection_s(args, world)
    mem_ok = free >= need
    time_ok = left >= 2 * proj
    ok = agree(mem_ok and time_ok, world)
    info = {"budget_s": args.budget_s, "elapsed_s": round(time.perf_counter() - T_START, 1),
            "projected_s": round(proj, 1), "rank0_free_device_bytes": free, "rank0_need_device_bytes": need,
            "device_total_bytes": total}
    if ok:
        return None, info
    why = []
    if not time_ok:
        why.append(f"projected {proj:.0f} s (x2 margin) past the {left:.0f} s left of --budget-s {args.budget_s}")
    if not mem_ok:
        why.append(f"rank {rank}: {free / 2**30:.1f} GiB free device memory < {need / 2**30:.1f} GiB needed")
    return ("; ".join(why) or "another rank lacks the device memory or time for C5"), info


def rccl_group(world, backend="nccl"):
    """The data-path process group over RCCL (torch.distributed backend "nccl" on ROCm).  World > 1:
    a new nccl group beside the gloo control-plane group dist_init made (backend "gloo": the
    rehearsal's stand-in when ranks share GPUs).  World 1: a one-rank nccl group of its own (RCCL
    still runs the scatter / gather: a one-rank communicator), so the RCCL path is exercised on a
    one-GPU box too."""
    import datetime
    import torch.distributed as dist
    # a collective that never completes (a rank that failed before it) ends the job at this
    # timeout; 120 s bounds what a broken leg costs the driver's scaling run
    to = datetime.timedelta(seconds=120)
    if world > 1:
        return dist.new_group(backend=backend, timeout=to)
    if not dist.is_initialized() and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") and os.environ.get("MASTER_PORT"):
        # one rank under torchrun: its tcp:// store would be a client of the agent's store, so take
        # torchrun's rendezvous (env://) instead of a private port
        dist.init_process_group("nccl", rank=0, world_size=1, timeout=to)
    if not dist.is_initialized():
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, timeout=to)
    return dist.group.WORLD


def rccl_c2_leg(args, rank, local, world, total, steps, warmup, eng=None, dump="", transport="nccl"):
    """Strong scaling over RCCL (BASELINE configs[4]'s batch scatter): ONE batch of
    `total` C2 pairs generated on rank 0 and resident on GPU 0 in the engine's 2-bit wire form
    (shards.BatchScatter: contiguous ranges of equal static band cells, each cut into
    --rccl-chunks pieces packed by bsw_pack_batch, ~134 B per pair), SCATTERED chunk by chunk to the
    ranks' GPUs by RCCL (every chunk's scatter issued at once), each piece scored in place as soon
    as it lands (bsw_get_scores_packed_device on its own stream and thread, so pieces overlap on
    the device), the 24 output bytes per pair GATHERED back to GPU 0 by RCCL chunk by chunk -- all
    inside the timed region (barrier + device sync on both sides, max over ranks).  Rank 0 then
    runs the whole batch alone on GPU 0 (bsw_get_scores_device on the resident batch: the one-GPU
    time of the same job, and the check that the gathered outputs are identical to it).
    A rank whose scoring fails keeps taking part in every collective and the ranks agree on the
    outcome over gloo afterwards (one rank must not leave the others blocked in RCCL).
    transport "gloo" (the --rehearse run, ranks sharing GPUs): the same steps with a gloo group over
    host buffers, each piece copied to the GPU to be scored and its outputs copied back -- labelled,
    never a scaling measurement.  Returns the leg's dict on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    import shards
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    g = rccl_group(world, "nccl" if transport == "nccl" else "gloo")
    wire_dev = dev if transport == "nccl" else torch.device("cpu")
    meta_g = dist.group.WORLD if world > 1 else None
    cfg = bsw.synth_cfg(h0_hi=args.h0_hi)
    t0 = time.perf_counter()
    pairs = ref = qer = None
    err = None
    if rank == 0:
        try:
            pairs, ref, qer = bsw.synth_batch(total, cfg=cfg)
        except Exception as e:  # noqa: BLE001
            err = e
    if not agree(err is None, world):
        return {"error": f"batch generation failed: {err!r}"[:400]} if rank == 0 else None
    bs = shards.BatchScatter(rank, world, g, wire_dev, pairs, ref, qer, w=args.w, meta_group=meta_g,
                             chunks=args.rccl_chunks)
    setup_s = time.perf_counter() - t0
    own = eng is None
    if own:
        eng = bsw.Engine(device=local)

    def score(c, recv, row, out):
        if transport == "nccl":
            eng.get_scores_packed_device(recv.data_ptr(), bsw.Packed.from_row(row), args.w, args.cell_bits,
                                         out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
            return
        r_d = recv.to(dev)                                   # rehearsal: host-staged piece
        o_d = torch.empty(out.shape, dtype=out.dtype, device=dev)
        eng.get_scores_packed_device(r_d.data_ptr(), bsw.Packed.from_row(row), args.w, args.cell_bits,
                                     o_d.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        out.copy_(o_d.cpu())

    for _ in range(warmup):
        bs.step(score)
    for k in bs.ms:
        bs.ms[k].clear()
    barrier(world)
    t = time.perf_counter()
    for _ in range(steps):
        bs.step(score)
    barrier(world)
    dt = time.perf_counter() - t
    dt_max = allreduce_max(dt, world)
    ok = bs.agree_ok()
    phase = {k: allreduce_max(float(np.mean(v)), world) for k, v in bs.ms.items()}
    rws = dist.get_world_size(g)
    if rank != 0:
        if own:
            eng.close()
        return None
    if not ok:
        return {"error": f"a rank's scoring failed: {bs.error!r}"[:400] if bs.error else "a rank's scoring failed",
                "rccl_world_size": rws}
    res = bs.merged()
    if dump:
        np.save(dump, res)
    # the same batch on GPU 0 alone: the one-GPU time of this job and the identity check
    d_p, d_r, d_q = (hiprt.DeviceBuffer.from_array(a) for a in (pairs, ref, qer))
    one = []
    for _ in range(3):
        d_p.upload(pairs)
        t = time.perf_counter()
        eng.get_scores_device(d_p.ptr, d_r.ptr, d_q.ptr, total, args.w, args.cell_bits)
        one.append(time.perf_counter() - t)
    single = d_p.download(np.empty_like(pairs))
    for b in (d_p, d_r, d_q):
        b.free()
    same = all(np.array_equal(res[f], single[f]) for f in bsw.OUT_FIELDS)
    if own:
        eng.close()
    ms = dt_max / steps * 1e3
    one_ms = statistics.median(one) * 1e3
    return {
        "value": round(total * steps / dt_max / 1e6, 3), "unit": UNIT, "scaling": "strong",
        "ms_per_step": round(ms, 3), "steps": steps, "warmup": warmup,
        "total_pairs": total, "pairs_rank0": bs.n_me, "chunks": bs.chunks,
        "wire_bytes_per_pair": round(bs.wire_bytes / total, 1), "shard_buffer_bytes": bs.S,
        "rccl_world_size": rws, "backend": dist.get_backend(g),
        **({} if transport == "nccl" else
           {"rehearsal": "gloo over host-staged buffers: ranks share GPUs, not a scaling measurement"}),
        "phase_ms_max_over_ranks": {k: round(v, 3) for k, v in phase.items()},
        "single_gpu_ms": round(one_ms, 3), "single_gpu_value": round(total / (one_ms * 1e-3) / 1e6, 3),
        "strong_speedup_vs_single_gpu": round(one_ms / ms, 3),
        "outputs_identical_to_single_gpu": bool(same),
        "setup_s": round(setup_s, 2),
        "step": "RCCL scatter of every chunk's 2-bit wire-form pieces from GPU 0 (issued at once) -> "
                "bsw_get_scores_packed_device on each piece as it lands (own stream per chunk) -> RCCL "
                "gather of 24 output bytes per pair to GPU 0 per chunk (all timed)",
    }


def main_strong_rccl(args, rank, local, world):
    """C5 as BASELINE configs[4] words it, as its own line: rccl_c2_leg over --total-pairs pairs,
    value = total pairs / max-over-ranks step time (scaling "strong")."""
    leg = rccl_c2_leg(args, rank, local, world, args.total_pairs, args.steps, args.warmup, dump=args.dump)
    if rank != 0:
        return
    if "value" not in leg:
        raise SystemExit(f"bench.py: the RCCL leg failed: {leg}")
    cfg = bsw.synth_cfg(h0_hi=args.h0_hi)
    N = args.total_pairs
    out_j = {
        "metric": METRIC, "value": leg.pop("value"), "unit": UNIT, "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": leg.pop("ms_per_step"), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int16", "data": "synthetic (bsw_synth.c, seed 42)",
        "config": {"workload": f"C5 strong scaling, RCCL batch scatter: one batch of {N} C2 pairs ({cfg.qlen} bp "
                               f"query / {cfg.tlen} bp ref, w={args.w}) resident on GPU 0, split over {world} "
                               f"rank(s) by static band cells, scattered / gathered with RCCL over xGMI inside "
                               f"the timed region",
                   "total_pairs": N, "pairs_rank0": leg["pairs_rank0"], "shard_buffer_bytes": leg["shard_buffer_bytes"],
                   "parallelism": f"split{world} (bsw_split_by_cells; RCCL scatter + gather)",
                   "distinct_gpus": args.distinct_gpus},
        "rccl": leg,
    }
    print(json.dumps(out_j), flush=True)


def mem_reference(ref_mb: int) -> np.ndarray:
    """main_mem's C4 reference: bsw_synth.c random bases, N -> a random base (bwa's .pac)"""
    ref = bsw.synth_reference(ref_mb * 1_000_000, seed=7)
    nb = ref > 3
    ref[nb] = np.random.default_rng(1).integers(0, 4, int(nb.sum()), dtype=np.uint8)
    return ref


class MemFrontEnd:
    """One rank's GPU front end over reads already in HBM: bsw_mem_collect_intv_device (SMEM
    seeding) -> bsw_mem_chain_device (SA lookups, mem_chain, mem_chain_flt) ->
    bsw_chain2aln_resident (mem_chain2aln against the resident two-strand text).  Device
    buffers are torch tensors; run() returns (seeds, extensions) and leaves the results in
    self.o[...] (seeds / sr / sc / out / ext, the first `seeds` entries valid)."""

    def __init__(self, fmi, eng, opt, n, cap, dev, seeds_cap):
        import torch
        self.torch, self.fmi, self.eng, self.opt, self.n, self.cap, self.dev = torch, fmi, eng, opt, n, cap, dev
        self.mopt, self.copt = bsw.mem_opt(), bsw.chain_opt()
        self.mems = torch.empty(max(1, n * cap * bsw.BWTINTV_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        self.cnt = torch.empty(max(1, n * 4), dtype=torch.uint8, device=dev)
        self.alloc(seeds_cap)

    def alloc(self, m):
        t = self.torch
        self.m = m
        self.o = {k: t.empty(max(1, m * sz), dtype=t.uint8, device=self.dev)
                  for k, sz in (("seeds", bsw.SEED_DTYPE.itemsize), ("sr", 4), ("sc", 4),
                                ("out", bsw.ALNREG_DTYPE.itemsize), ("ext", 4))}

    def run(self, p_reads, p_off, p_len, grow=True):
        P = {k: v.data_ptr() for k, v in self.o.items()}
        bsw._check(self.fmi.collect_intv_device(p_reads, p_off, p_len, self.n, 150, self.mems.data_ptr(), self.cap,
                                                self.cnt.data_ptr(), self.mopt))
        rc, ns = self.fmi.mem_chain_device(p_len, self.n, self.mems.data_ptr(), self.cap, self.cnt.data_ptr(),
                                           P["seeds"], P["sr"], P["sc"], self.m, self.copt)
        if rc == -34:                                    # more seeds than room (sizing passes only)
            if not grow:
                raise RuntimeError(f"{ns} seeds past the capacity {self.m} inside the timed region")
            self.alloc(int(ns * 1.25) + 16)
            return self.run(p_reads, p_off, p_len, grow=False)
        bsw._check(rc)
        bsw.chain2aln_resident(self.eng, p_reads, p_off, p_len, self.n, P["seeds"], P["sr"], P["sc"], ns,
                               P["out"], P["ext"], self.opt)
        hiprt.synchronize()
        return ns, sum(bsw.chain_last_stats(self.eng).n_pairs)

    def pack(self, ns, rec):
        """rec[:ns] = shards.REC_DTYPE rows (17 int32 per seed), on the device"""
        t = self.torch
        i32 = lambda k, w: self.o[k][:ns * 4 * w].view(t.int32).view(ns, w)   # noqa: E731
        rec[:ns, 0:4] = i32("seeds", 4)
        rec[:ns, 4:5] = i32("sr", 1)
        rec[:ns, 5:6] = i32("sc", 1)
        rec[:ns, 6:16] = i32("out", 10)
        rec[:ns, 16:17] = i32("ext", 1)

    def records(self, ns) -> np.ndarray:
        import shards
        rec = self.torch.zeros((max(1, ns), shards.REC_WORDS), dtype=self.torch.int32, device=self.dev)
        self.pack(ns, rec)
        return np.ascontiguousarray(rec[:ns].cpu().numpy()).view(shards.REC_DTYPE).reshape(-1)


def agree(ok: bool, world: int) -> bool:
    """gloo all-reduce of a success flag: True only when every rank's `ok` is (ranks decide
    together whether to enter the next RCCL phase, so none is left blocked in a collective)"""
    if world == 1:
        return ok
    import torch
    import torch.distributed as dist
    t = torch.tensor([0 if ok else 1], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item()) == 0


def rccl_c5_leg(args, rank, local, world, n_reads, ref_mb, steps, warmup, dump="", blocks_only=False):
    """C5 as BASELINE configs[4] words it, on the full front end: ONE set of n_reads PE reads
    generated on rank 0 and resident on GPU 0, cut into contiguous read ranges and SCATTERED to the
    ranks' GPUs by RCCL (shards.ReadScatter); every rank runs SMEM seeding -> chaining ->
    mem_chain2aln on its shard against its own index of the ref_mb reference (built on its GPU
    before timing); every seed's record (seed, read, chain, region, extended flag: 68 B) is
    GATHERED back to GPU 0 by RCCL.  Scatter, front end and gather are timed (barrier + sync on
    both sides, max over ranks).  Rank 0 then runs the whole read set alone on GPU 0: the one-GPU
    time of the same job and the check that the gathered records are identical to it.  Ranks
    agree over gloo before the first RCCL collective (a rank whose setup failed makes every rank
    skip the leg) and after the timed steps (a failed front end is held, never left hanging).
    Returns the leg's dict on rank 0 (an "error" entry if it failed), None elsewhere."""
    import torch
    import torch.distributed as dist
    import shards
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    t0 = time.perf_counter()
    log = lambda m: print(f"[bench c5 rank {rank}] {m} ({time.perf_counter() - t0:.1f} s)",  # noqa: E731
                          file=sys.stderr, flush=True)
    err = None
    try:
        ref = mem_reference(ref_mb)
        reads = off = lens = None
        if rank == 0:
            reads, off, lens = pe_reads(ref, max(1, n_reads // 2), seed=42)
        gen_s = time.perf_counter() - t0
        t = time.perf_counter()
        fmi = bsw.Fmi(ref, device=local, flags=(bsw.FMI_NO_TEXT if blocks_only else None))
        build_s = time.perf_counter() - t
        eng = bsw.Engine(device=local)
        T = np.concatenate([ref, (3 - ref[::-1])]).astype(np.uint8)
        bsw.set_reference(eng, T)
        del T
        l_pac = len(ref)
    except Exception as e:  # noqa: BLE001
        err = e
    meta_g = dist.group.WORLD if world > 1 else None
    if not agree(err is None, world):
        return {"error": f"setup failed on a rank: {err!r}"[:400] if err else "setup failed on another rank"} \
            if rank == 0 else None
    g = rccl_group(world)
    rs = shards.ReadScatter(rank, world, g, dev, reads, off, lens, meta_group=meta_g)
    N = int(rs.meta[:, 0].sum())
    log(f"{N} reads, {rs.n_me} on this rank; index built in {build_s:.1f} s")
    opt = bsw.ext_opt(w=args.w, l_pac=l_pac)
    cap = 256 if N <= 2_000_000 else 64                  # as one GPU would run the whole set (main_mem)
    fe = MemFrontEnd(fmi, eng, opt, rs.n_me, cap, dev, max(16, 4 * rs.n_me))
    o_reads, o_off, o_len = rs.layout()

    def score(recv, row, rec):
        base = recv.data_ptr()
        ns, ne = fe.run(base + o_reads, base + o_off, base + o_len, grow=rec is None)
        score.n_ext += ne
        if rec is not None:
            fe.pack(ns, rec)
        return ns
    score.n_ext = 0
    # sizing pass (untimed): the seed count fixes the gathered record capacity
    rs.scatter()
    try:
        ns0 = score(rs.recv, rs.meta[rank], None) if rs.n_me > 0 else 0
    except Exception as e:  # noqa: BLE001
        err, ns0 = e, 0
    rs.size(ns0 + 16)
    if not agree(err is None, world):
        fmi.close()
        return {"error": f"sizing pass failed on a rank: {err!r}"[:400] if err else "sizing failed on another rank"} \
            if rank == 0 else None
    for _ in range(warmup):
        rs.step(score)
    for k in rs.ms:
        rs.ms[k].clear()
    score.n_ext = 0
    barrier(world)
    t = time.perf_counter()
    for _ in range(steps):
        rs.step(score)
    barrier(world)
    dt = time.perf_counter() - t
    dt_max = allreduce_max(dt, world)
    ok = rs.agree_ok()
    n_ext_all = allreduce_sum(score.n_ext, world)
    phase = {k: allreduce_max(float(np.mean(v)), world) for k, v in rs.ms.items()}
    rws = dist.get_world_size(g)
    if rank != 0:
        fmi.close()
        return None
    if not ok:
        fmi.close()
        return {"error": f"a rank's front end failed: {rs.error!r}"[:400] if rs.error else "a rank's front end failed",
                "rccl_world_size": rws}
    got = rs.merged()
    if dump:
        np.save(dump, got)
    # the whole read set on GPU 0 alone (its own buffers; same index and engine)
    d_r = torch.from_numpy(reads).to(dev)
    d_o = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_l = torch.from_numpy(lens.astype(np.int32)).to(dev)
    del fe
    one_fe = MemFrontEnd(fmi, eng, opt, N, cap, dev, max(16, 4 * N))
    one = []
    for k in range(3):
        t = time.perf_counter()
        ns1, _ = one_fe.run(d_r.data_ptr(), d_o.data_ptr(), d_l.data_ptr(), grow=(k == 0))
        one.append(time.perf_counter() - t)
    want = one_fe.records(ns1)
    same = bool(len(want) == len(got) and np.array_equal(want.view(np.uint8), got.view(np.uint8)))
    fmi.close()
    ms = dt_max / steps * 1e3
    one_ms = statistics.median(one[1:]) * 1e3
    return {
        "value": round(n_ext_all / dt_max / 1e6, 3), "unit": UNIT, "scaling": "strong",
        "ms_per_step": round(ms, 3), "steps": steps, "warmup": warmup,
        "reads_per_s_M": round(N * steps / dt_max / 1e6, 3),
        "total_reads": N, "reads_rank0": rs.n_me, "ref_bases": int(l_pac),
        "rccl_world_size": rws, "backend": dist.get_backend(g), "shard_buffer_bytes": rs.S,
        "record_bytes_per_seed": shards.REC_DTYPE.itemsize, "record_capacity": rs.cap,
        "phase_ms_max_over_ranks": {k: round(v, 3) for k, v in phase.items()},
        "seeds": int(len(got)),
        "single_gpu_ms": round(one_ms, 3), "strong_speedup_vs_single_gpu": round(one_ms / ms, 3),
        "outputs_identical_to_single_gpu": same,
        "index_build_s": round(build_s, 2), "synth_gen_s": round(gen_s, 2),
        "step": "RCCL scatter of the PE read shards from GPU 0 -> every rank: SMEM seeding -> SA + mem_chain + "
                "mem_chain_flt -> mem_chain2aln on its own GPU-resident index -> RCCL gather of the per-seed "
                "records to GPU 0 (all timed)",
    }


def main_mem_strong_rccl(args, rank, local, world):
    """C5 as its own line (--workload c4mem --scaling strong --transport rccl): rccl_c5_leg over
    --reads PE reads vs a --ref-mb reference; value = extensions / max-over-ranks step time."""
    leg = rccl_c5_leg(args, rank, local, world, args.reads, args.ref_mb, args.steps, args.warmup, dump=args.dump,
                      blocks_only=args.fmi_blocks_only)
    if rank != 0:
        return
    if "value" not in leg:
        raise SystemExit(f"bench.py: the C5 leg failed: {leg}")
    N = leg["total_reads"]
    out_j = {
        "metric": METRIC, "value": leg.pop("value"), "unit": UNIT, "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": leg.pop("ms_per_step"), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int16",
        "data": "synthetic PE reads (bench.pe_reads) from a bsw_synth.c random reference",
        "config": {"workload": f"C5 strong scaling, RCCL read scatter: one set of {N} PE 150 bp reads resident on "
                               f"GPU 0 vs a {args.ref_mb} Mb random reference, split over {world} rank(s), "
                               f"scattered with RCCL over xGMI; every rank: FM-index SMEM seeding -> SA + mem_chain "
                               f"+ mem_chain_flt -> mem_chain2aln on its own GPU-resident index; per-seed records "
                               f"gathered to GPU 0 with RCCL, inside the timed region",
                   "total_reads": N, "reads_rank0": leg["reads_rank0"], "ref_bases": leg["ref_bases"],
                   "parallelism": f"split{world} (contiguous read ranges; RCCL scatter + gather)",
                   "distinct_gpus": args.distinct_gpus},
        "reads_per_s_M": leg["reads_per_s_M"],
        "rccl": {k: leg[k] for k in ("rccl_world_size", "backend", "shard_buffer_bytes", "record_bytes_per_seed",
                                     "record_capacity", "phase_ms_max_over_ranks")},
        "seeds": leg["seeds"],
        "single_gpu_ms": leg["single_gpu_ms"], "strong_speedup_vs_single_gpu": leg["strong_speedup_vs_single_gpu"],
        "outputs_identical_to_single_gpu": leg["outputs_identical_to_single_gpu"],
        "index_build_s": leg["index_build_s"], "synth_gen_s": leg["synth_gen_s"],
    }
    print(json.dumps(out_j), flush=True)


def main_strong(args, rank, local, world):
    """C5-shaped strong scaling: ONE batch of --total-pairs C2 pairs (the whole job), split over
    the ranks into contiguous ranges of equal static band cells (bsw_split_by_cells, SURVEY.md
    §8(e)).  Every rank holds its range in host memory, as the process that built the batch
    would; a step = bsw_get_scores on those HOST buffers (pinned chunked pipeline: H2D over the
    rank's own PCIe link, plan / sort / DP, D2H of the records) -- the distribution and the
    gather are inside the timed region.  value = total pairs / max-over-ranks step time."""
    cfg = bsw.synth_cfg(h0_hi=args.h0_hi)
    N = args.total_pairs
    t0 = time.perf_counter()
    meta = np.zeros(N, dtype=bsw.SEQPAIR_DTYPE)          # lengths of the whole batch (for the cut)
    step_n = 1_000_000
    for a in range(0, N, step_n):
        m = min(step_n, N - a)
        meta[a:a + m] = bsw.synth_batch(m, pair_base=a, cfg=cfg)[0]
    cut = bsw.split_by_cells(meta, args.w, world)
    lo, hi = int(cut[rank]), int(cut[rank + 1])
    del meta
    # the rank's range as host batches of <= 2M pairs (SeqPair idr / idq are int32 offsets
    # into one call's buffers, so one getScores call cannot address more than 2 GB of bases)
    piece = 2_000_000
    batches = [bsw.synth_batch(min(piece, hi - a), pair_base=a, cfg=cfg) for a in range(lo, hi, piece)]
    gen_s = time.perf_counter() - t0
    eng = bsw.Engine(device=local)

    def step():
        for p, r, q in batches:
            eng.get_scores(p, r, q, args.w, args.cell_bits)

    for _ in range(args.warmup):
        step()
    barrier(world)
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier(world)
    dt = time.perf_counter() - t
    dt_max = allreduce_max(dt, world)
    kms = eng.last_stats().kernel_ms
    kms_max = allreduce_max(kms, world)
    if args.dump:
        import torch
        import torch.distributed as dist
        work = np.concatenate([b[0] for b in batches]) if batches else np.zeros(0, bsw.SEQPAIR_DTYPE)
        out = torch.from_numpy(work.view(np.int32).reshape(-1, 14).copy())
        if world > 1:
            sizes = [int(cut[r + 1] - cut[r]) for r in range(world)]
            gathered = [torch.zeros((sz, 14), dtype=torch.int32) for sz in sizes] if rank == 0 else None
            dist.gather(out, gathered, dst=0)
        else:
            gathered = [out]
        if rank == 0:
            np.save(args.dump, np.concatenate([g.numpy() for g in gathered]).view(bsw.SEQPAIR_DTYPE).reshape(-1))
    if rank != 0:
        return
    value = N * args.steps / dt_max / 1e6
    out_j = {
        "metric": METRIC, "value": round(value, 3), "unit": UNIT, "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int16", "data": "synthetic (bsw_synth.c, seed 42)",
        "config": {"workload": f"C5 strong scaling: one batch of {N} C2 pairs ({cfg.qlen} bp query / {cfg.tlen} bp "
                               f"ref, w={args.w}) split over {world} rank(s) by static band cells; host buffers, "
                               f"PCIe H2D + D2H inside the timed region",
                   "total_pairs": N, "pairs_rank0": hi - lo, "cut": [int(c) for c in cut],
                   "parallelism": f"split{world} (bsw_split_by_cells, no data-path collective)",
                   "distinct_gpus": args.distinct_gpus},
        "dp_kernel_ms_last_call_max_over_ranks": round(kms_max, 3),
        "host_batches_rank0": len(batches),
        "synth_gen_s": round(gen_s, 2),
    }
    if args.distinct_gpus < world:
        out_j["rehearsal"] = f"{world} ranks on {args.distinct_gpus} GPU(s): not a scaling measurement"
    print(json.dumps(out_j), flush=True)


def main_c4(args, rank, local, world):
    """C4/C5-shaped run of the extension pipeline (include/bsw_ext.h): per GPU `--reads` 150 bp
    reads sampled from a random reference, one exact seed each (what upstream's host SMEM seeding
    hands to mem_chain2aln).  The reference is RESIDENT in HBM (bsw_set_reference) and the reads
    and seeds are in HBM when the timed region starts; a step = bsw_extend_seeds_device over the
    rank's reads: job building, LEFT batch (+ band retries), interpretation, RIGHT batch
    (+ retries), interpretation -- all on the GPU.  Reported as extensions/s (SeqPairs through the
    engine) and reads/s; beside it the PCIe-inclusive rate (reads up, regions down) and the
    host-built pipeline (bsw_extend_seeds).  FM-index seeding is out of scope (the
    north star keeps it on the host); extension cost does not depend on the reference size."""
    t0 = time.perf_counter()
    ref = bsw.synth_reference(args.ref_mb * 1_000_000, seed=7)
    exact = getattr(args, "exact", False)
    rcfg = bsw.reads_cfg(p_sub=0.0, p_indel=0.0, p_unrelated=0.0) if exact else None
    reads, off, lens, seeds, _ = bsw.synth_reads(ref, args.reads, read_base=rank * args.reads, cfg=rcfg)
    gen_s = time.perf_counter() - t0
    eng = bsw.Engine(device=local)
    opt = bsw.ext_opt(w=args.w)
    bsw.set_reference(eng, ref)
    d_in = [hiprt.DeviceBuffer.from_array(a) for a in (reads, off, lens, seeds)]
    out = np.zeros(args.reads, dtype=bsw.ALNREG_DTYPE)
    d_out = hiprt.DeviceBuffer(out.nbytes)

    def step():
        bsw.extend_seeds_device(eng, d_in[0].ptr, d_in[1].ptr, d_in[2].ptr, d_in[3].ptr, args.reads, d_out.ptr, opt)
        st = bsw.ext_last_stats(eng)
        return sum(st.n_pairs), st.kernel_ms

    for _ in range(args.warmup):
        step()
    barrier(world)
    t = time.perf_counter()
    n_ext, kms = 0, []
    for _ in range(args.steps):
        ne, km = step()
        n_ext += ne
        kms.append(km)
    barrier(world)
    dt = time.perf_counter() - t
    dt_max = allreduce_max(dt, world)
    n_ext_all = allreduce_sum(n_ext, world)
    d_out.download(out)
    if rank != 0:
        return
    st = bsw.ext_last_stats(eng)
    value = n_ext_all / dt_max / 1e6
    # PCIe-inclusive (reads + seeds up, regions down; resident reference) and host-built rates
    t = time.perf_counter()
    reg_res = bsw.extend_seeds_resident(eng, reads, off, lens, seeds, opt)
    pcie_s = time.perf_counter() - t
    t = time.perf_counter()
    reg_host = bsw.extend_seeds(eng, ref, reads, off, lens, seeds, opt)
    host_s = time.perf_counter() - t
    hst = bsw.ext_last_stats(eng)
    same = all(np.array_equal(reg_res[f], out[f]) and np.array_equal(reg_host[f], out[f])
               for f in bsw.ALNREG_DTYPE.names)
    if exact:     # exact reads: the seed is the whole read, no extension runs -> report reads/s
        value = args.reads * world * args.steps / dt_max / 1e6
    out_j = {
        "metric": "M reads/sec through the extension pipeline (C1 plumbing: exact reads)" if exact else METRIC,
        "value": round(value, 3), "unit": "M reads/s" if exact else UNIT, "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int16", "data": "synthetic (bsw_synth.c reads, seed 42)",
        "config": {"workload": ("C1-shaped (exact reads, plumbing): " if exact else "C4-shaped extension pipeline: ") +
                               f"{args.reads} x 150 bp reads/GPU from a "
                               f"{args.ref_mb} Mb random reference resident in HBM, one exact seed each, "
                               f"LEFT+RIGHT extensions w={args.w} with band retry, job build and "
                               f"interpretation on the GPU, reads resident in HBM",
                   "reads_per_gpu": args.reads, "parallelism": f"shard{world} (independent reads)",
                   "extensions_per_step_rank0": list(st.n_pairs)},
        "reads_per_s_M": round(args.reads * world * args.steps / dt_max / 1e6, 3),
        "dp_kernel_ms_per_step": round(float(np.mean(kms)), 3),
        "pcie_inclusive_reads_per_s_M": round(args.reads / pcie_s / 1e6, 3),
        "host_built_pipeline": {"reads_per_s_M": round(args.reads / host_s / 1e6, 3),
                                "build_ms": round(hst.build_ms, 2), "engine_incl_pcie_ms": round(hst.engine_ms, 2),
                                "interpret_ms": round(hst.interp_ms, 2)},
        "device_host_paths_identical": bool(same),
        "to_end_fraction": round(float(np.mean((out["qb"] == 0) & (out["qe"] == lens))), 4),
    }
    if world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # CPU baseline leg only (test infrastructure)
        S = min(args.reads, 20_000)
        t = time.perf_counter()
        ref_reg = oracle.extend_seeds(oracle.make_params(), opt, ref, reads, off[:S], lens[:S], seeds[:S])
        dt_cpu = time.perf_counter() - t
        n_cpu = int(np.sum((seeds[:S]["len"] > 0) & (seeds[:S]["qbeg"] > 0)) +
                    np.sum((seeds[:S]["len"] > 0) & (seeds[:S]["qbeg"] + seeds[:S]["len"] < lens[:S])))
        out_j["cpu_baseline"] = {
            "value": round((S if exact else n_cpu) / dt_cpu / 1e6, 4), "unit": "M reads/s" if exact else UNIT,
            "cores": 1, "kind": "port",
            "sample": f"first {S} reads; oracle/ext_ref.c (per-read mem_chain2aln extension restated, "
                      f"scalar ksw_extend2), 1 thread; first-try extensions counted",
            "outputs_identical_to_gpu": bool(all(np.array_equal(ref_reg[f], out[:S][f])
                                                 for f in bsw.ALNREG_DTYPE.names)),
        }
    out_j["synth_gen_s"] = round(gen_s, 2)
    print(json.dumps(out_j), flush=True)


def main_c4pe(args, rank, local, world):
    """C4/C5: `--reads` paired-end 150 bp reads per GPU (reads/2 fragments, insert 400-600) from a
    `--ref-mb` random reference RESIDENT in HBM, with every maximal exact run >= 19 bp along each
    read's true path as a seed (one chain, longest first) plus a planted spurious chain on 10%
    of the reads (bsw_synth_pe_seeds).  A step = bsw_chain2aln_device over all of them: upstream's
    per-read chain / seed order with contained-seed skipping (mem_chain2aln), batched across reads
    in rounds; each round's LEFT / RIGHT extensions (+ band retries) run on the GPU against the
    resident reads and reference.  Reported: extensions/s (SeqPairs through the engine) and
    reads/s; seeds per read, extended fraction and rounds beside it.  FM-index seeding is out of
    scope (the north star keeps it on the host)."""
    t0 = time.perf_counter()
    ref = bsw.synth_reference(args.ref_mb * 1_000_000, seed=7)
    npairs = max(1, args.reads // 2)
    reads, off, lens, seeds, sr, sc = bsw.synth_pe_seeds(ref, npairs, pair_base=rank * npairs)
    gen_s = time.perf_counter() - t0
    eng = bsw.Engine(device=local)
    opt = bsw.ext_opt(w=args.w)
    bsw.set_reference(eng, ref)
    d_reads = hiprt.DeviceBuffer.from_array(reads)

    out_buf = np.zeros(len(seeds), dtype=bsw.ALNREG_DTYPE)
    ext_buf = np.zeros(len(seeds), dtype=np.int32)
    # everything resident in HBM before timing (value); the host-array form is timed beside it
    d_in = {k: hiprt.DeviceBuffer.from_array(v) for k, v in dict(off=off, lens=lens, seeds=seeds, sr=sr, sc=sc).items()}
    d_out = hiprt.DeviceBuffer(len(seeds) * bsw.ALNREG_DTYPE.itemsize)
    d_ext = hiprt.DeviceBuffer(len(seeds) * 4)

    def step():
        bsw.chain2aln_resident(eng, d_reads.ptr, d_in["off"].ptr, d_in["lens"].ptr, len(lens), d_in["seeds"].ptr,
                               d_in["sr"].ptr, d_in["sc"].ptr, len(seeds), d_out.ptr, d_ext.ptr, opt)
        st = bsw.chain_last_stats(eng)
        return None, None, st

    for _ in range(args.warmup):
        step()
    barrier(world)
    t = time.perf_counter()
    n_ext, sts = 0, []
    for _ in range(args.steps):
        out, ext, st = step()
        n_ext += sum(st.n_pairs)
        sts.append(st)
    barrier(world)
    dt = time.perf_counter() - t
    dt_max = allreduce_max(dt, world)
    n_ext_all = allreduce_sum(n_ext, world)
    out = d_out.download(out_buf)
    ext = d_ext.download(ext_buf)
    if args.dump:                                    # every rank: its shard's regions (tests)
        np.savez(f"{args.dump}.rank{rank}.npz", out=out, ext=ext)
    # the host-array form (bsw_chain2aln_device: seeds up, regions down inside the call)
    t = time.perf_counter()
    for _ in range(2):
        h_out, h_ext = bsw.chain2aln_device(eng, d_reads.ptr, off, lens, seeds, sr, sc, opt)
    dt_host = (time.perf_counter() - t) / 2
    same_forms = bool(np.array_equal(h_ext, ext) and all(np.array_equal(h_out[f], out[f]) for f in bsw.ALNREG_DTYPE.names))
    if rank != 0:
        return
    st = sts[-1]
    value = n_ext_all / dt_max / 1e6
    nreads = 2 * npairs
    out_j = {
        "metric": METRIC, "value": round(value, 3), "unit": UNIT, "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int16", "data": "synthetic (bsw_synth.c PE reads, seed 42)",
        "config": {"workload": f"C4: {nreads} paired-end 150 bp reads/GPU ({npairs} fragments, insert 400-600) from a "
                               f"{args.ref_mb} Mb random reference resident in HBM, {len(seeds)} seeds "
                               f"({len(seeds) / nreads:.2f}/read, chains of every exact run >= 19 bp + 10% spurious "
                               f"chains), mem_chain2aln with contained-seed skipping, w={args.w}, band retry",
                   "reads_per_gpu": nreads, "parallelism": f"shard{world} (independent reads)",
                   "distinct_gpus": args.distinct_gpus},
        "reads_per_s_M": round(nreads * world * args.steps / dt_max / 1e6, 3),
        "seeds_per_read": round(len(seeds) / nreads, 3),
        "extended_fraction": round(st.n_extended / max(1, len(seeds)), 4),
        "rounds": st.rounds,
        "extensions_per_step_rank0": list(st.n_pairs),
        "dp_kernel_ms_per_step": round(float(np.mean([x.kernel_ms for x in sts])), 3),
        "host_containment_ms_per_step": round(float(np.mean([x.check_ms for x in sts])), 3),
        "host_prep_ms_per_step": round(float(np.mean([x.prep_ms for x in sts])), 3),
        "extension_calls_ms_per_step": round(float(np.mean([x.ext_ms for x in sts])), 3),
        "step": "bsw_chain2aln_resident (reads, seeds, regions in HBM; chain order, containment and picks on "
                "the GPU, one job-count readback per round)",
        "host_arrays_value": round(sum(st.n_pairs) / dt_host / 1e6, 3),
        "host_arrays_note": "bsw_chain2aln_device: seeds / read table up and regions down inside each call",
        "host_arrays_identical": same_forms,
    }
    if world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # CPU baseline leg only (test infrastructure)
        nt = cpu_leg_threads()
        S1 = int(np.searchsorted(sr, min(nreads, 20_000)))    # seeds of the first 20K reads (1 thread)
        S = int(np.searchsorted(sr, min(nreads, 20_000 * nt)))
        t = time.perf_counter()
        oracle.chain2aln(oracle.make_params(), opt, ref, reads, off, lens, seeds[:S1], sr[:S1], sc[:S1])
        dt_1 = time.perf_counter() - t
        t = time.perf_counter()
        want, wext = oracle.chain2aln(oracle.make_params(), opt, ref, reads, off, lens, seeds[:S], sr[:S], sc[:S],
                                      nthreads=nt)
        dt_cpu = time.perf_counter() - t
        # the extensions the CPU ran: LEFT / RIGHT of every extended seed (+ retries not counted)
        n_ext_of = lambda k: int(np.sum(wext[:k] * ((seeds[:k]["qbeg"] > 0).astype(int) +   # noqa: E731
                                                   ((seeds[:k]["qbeg"] + seeds[:k]["len"]) < lens[sr[:k]]).astype(int))))
        n_cpu = n_ext_of(S)
        rate = n_cpu / dt_cpu / 1e6
        out_j["cpu_baseline"] = {
            "value": round(rate, 4), "unit": UNIT, "cores": nt, "kind": "port",
            "sample": f"seeds of the first {min(nreads, 20_000 * nt)} reads ({S}); oracle/ext_ref.c oracle_chain2aln "
                      f"(literal per-read mem_chain2aln, scalar ksw_extend2) on {nt} threads (reads split, "
                      f"oracle_chain2aln_mt); first-try extensions counted",
            "one_thread": round(n_ext_of(S1) / dt_1 / 1e6, 5),
            "per_core_rate": round(rate / nt, 5),
            "node_extrapolated": node_extrapolation(rate, nt),
            "host": host_cpu_info(),
            "outputs_identical_to_gpu": bool(np.array_equal(wext, ext[:S]) and
                                             all(np.array_equal(want[f], out[:S][f]) for f in bsw.ALNREG_DTYPE.names)),
        }
    out_j["synth_gen_s"] = round(gen_s, 2)
    print(json.dumps(out_j), flush=True)


def pe_reads(ref, npairs: int, L: int = 150, seed: int = 42, ins=(400, 600), p_sub=0.01, p_n=0.001):
    """npairs fragments (insert uniform in `ins`) from either strand of ref: read 2k from the
    fragment's start, read 2k+1 the reverse complement of its end; 1% substitutions, 0.1% N."""
    rng = np.random.default_rng(seed)
    ln = rng.integers(ins[0], ins[1] + 1, npairs)
    st = rng.integers(0, len(ref) - ins[1] - 1, npairs)
    a = ref[st[:, None] + np.arange(L)[None, :]]
    b = ref[(st + ln - L)[:, None] + np.arange(L)[None, :]]
    b = (3 - b[:, ::-1]).astype(np.uint8)
    flip = rng.random(npairs) < 0.5                     # fragment from the reverse strand
    a[flip], b[flip] = b[flip].copy(), a[flip].copy()
    reads = np.stack([a, b], axis=1).reshape(2 * npairs, L)
    sub = rng.random(reads.shape) < p_sub
    reads[sub] = ((reads[sub] + rng.integers(1, 4, int(sub.sum()))) % 4).astype(np.uint8)
    reads[rng.random(reads.shape) < p_n] = 4
    n = 2 * npairs
    return np.ascontiguousarray(reads).reshape(-1), np.arange(n, dtype=np.int64) * L, np.full(n, L, np.int32)


def main_mem(args, rank, local, world, c1: bool):
    """The GPU front end of mem_align1_core over resident reads: FM-index SMEM seeding
    (bsw_mem_collect_intv_device) -> SA lookups + chaining + chain filtering
    (bsw_mem_chain_device) -> mem_chain2aln with contained-seed skipping
    (bsw_chain2aln_resident) against the resident two-strand text (l_pac clamp).  c1: BASELINE
    configs[0] -- the reference's own 10K exact 150 bp SE reads vs its 1 Mb reference
    (bwa-mem2-arm_amd/py/c1data.py, regenerated bit-exactly); else C4: --reads PE reads vs a
    --ref-mb random reference.  The index is built on the host before timing (build time
    reported); a step = the three stages over every read, seeding time included."""
    import c1data
    t0 = time.perf_counter()
    if c1:
        ref, reads, off, lens, _ = c1data.workload()
    else:
        ref = bsw.synth_reference(args.ref_mb * 1_000_000, seed=7)
        nb = ref > 3                                     # bwa's .pac: N -> a random base
        ref[nb] = np.random.default_rng(1).integers(0, 4, int(nb.sum()), dtype=np.uint8)
        reads, off, lens = pe_reads(ref, max(1, args.reads // 2), seed=42 + rank)
    n = len(lens)
    gen_s = time.perf_counter() - t0
    log = lambda m: print(f"[bench c4mem rank {rank}] {m} ({time.perf_counter() - t0:.1f} s)", file=sys.stderr,  # noqa: E731
                          flush=True)
    log(f"generated {n} reads vs {len(ref)} bases")
    t = time.perf_counter()
    fmi = bsw.Fmi(ref, device=local, flags=(bsw.FMI_NO_TEXT if args.fmi_blocks_only else None))
    build_s = time.perf_counter() - t
    log(f"index built in {build_s:.1f} s")
    T = np.concatenate([ref, (3 - ref[::-1])]).astype(np.uint8)
    eng = bsw.Engine(device=local)
    bsw.set_reference(eng, T)
    opt = bsw.ext_opt(w=args.w, l_pac=len(ref))
    # BSW_BENCH_MEMOPT="max_mem_intv=0,split_factor=1000": seeding-option experiments (which pass
    # costs what); the line's config then says so -- never a headline setting
    mo_kw = {k: (float(v) if k == "split_factor" else int(v)) for k, v in
             (x.split("=") for x in os.environ.get("BSW_BENCH_MEMOPT", "").split(",") if x)}
    mopt, copt = bsw.mem_opt(**mo_kw), bsw.chain_opt()
    cap = 256 if n <= 2_000_000 else 64                  # interval slots per read (HBM: n * cap * 32 B)
    d_reads = hiprt.DeviceBuffer.from_array(reads)
    d_off, d_len = hiprt.DeviceBuffer.from_array(off), hiprt.DeviceBuffer.from_array(lens)
    d_mems = hiprt.DeviceBuffer(n * cap * bsw.BWTINTV_DTYPE.itemsize)
    d_cnt = hiprt.DeviceBuffer(n * 4)
    sc_cap = [max(16, 4 * n)]
    bufs = {}

    def alloc(m):
        bufs.update(seeds=hiprt.DeviceBuffer(m * bsw.SEED_DTYPE.itemsize), sr=hiprt.DeviceBuffer(m * 4),
                    sc=hiprt.DeviceBuffer(m * 4), out=hiprt.DeviceBuffer(m * bsw.ALNREG_DTYPE.itemsize),
                    ext=hiprt.DeviceBuffer(m * 4))
        sc_cap[0] = m
    alloc(sc_cap[0])

    def step():
        ta = time.perf_counter()
        bsw._check(fmi.collect_intv_device(d_reads.ptr, d_off.ptr, d_len.ptr, n, 150, d_mems.ptr, cap, d_cnt.ptr, mopt))
        tb = time.perf_counter()
        rc, ns = fmi.mem_chain_device(d_len.ptr, n, d_mems.ptr, cap, d_cnt.ptr, bufs["seeds"].ptr, bufs["sr"].ptr,
                                      bufs["sc"].ptr, sc_cap[0], copt)
        if rc == -34:                                    # more seeds than room: grow, redo (counted)
            alloc(int(ns * 1.25) + 16)
            rc, ns = fmi.mem_chain_device(d_len.ptr, n, d_mems.ptr, cap, d_cnt.ptr, bufs["seeds"].ptr,
                                          bufs["sr"].ptr, bufs["sc"].ptr, sc_cap[0], copt)
        bsw._check(rc)
        tc = time.perf_counter()
        bsw.chain2aln_resident(eng, d_reads.ptr, d_off.ptr, d_len.ptr, n, bufs["seeds"].ptr, bufs["sr"].ptr,
                               bufs["sc"].ptr, ns, bufs["out"].ptr, bufs["ext"].ptr, opt)
        td = time.perf_counter()
        smem_ms[0] = fmi.last_kernel_ms()
        return ns, bsw.chain_last_stats(eng), (tb - ta, tc - tb, td - tc)

    # --pipeline P: the reads in P batches; batch k's mem_chain2aln (engine streams) runs on a second
    # host thread while batch k + 1 is seeded and chained (the index's stream, one call at a time per
    # index).  Batch k's seeds go at seed offset soff_k of the shared buffers with batch-relative read
    # numbers; read b of the batch is read a_k + b of the step (d_off / d_len / d_mems / d_cnt offset).
    P = 1 if c1 else max(1, int(args.pipeline))
    bounds = [n * k // P for k in range(P + 1)]
    seg = []                                             # (a_k, soff_k, ns_k) of the last step
    smem_ms = [0.0]

    def step_pipe():
        import queue
        import threading
        q, res = queue.Queue(), {"st": [], "err": None, "t": 0.0}
        SZ, AZ, MZ = bsw.SEED_DTYPE.itemsize, bsw.ALNREG_DTYPE.itemsize, bsw.BWTINTV_DTYPE.itemsize

        def extender():
            while True:
                it = q.get()
                if it is None:
                    return
                a, b, so, nk = it
                if res["err"] is not None or nk == 0:
                    continue
                try:
                    t1 = time.perf_counter()
                    bsw.chain2aln_resident(eng, d_reads.ptr, d_off.ptr + 8 * a, d_len.ptr + 4 * a, b - a,
                                           bufs["seeds"].ptr + so * SZ, bufs["sr"].ptr + 4 * so,
                                           bufs["sc"].ptr + 4 * so, nk, bufs["out"].ptr + so * AZ,
                                           bufs["ext"].ptr + 4 * so, opt)
                    res["t"] += time.perf_counter() - t1
                    res["st"].append(bsw.chain_last_stats(eng))
                except Exception as e:  # noqa: BLE001 -- re-raised on the caller's thread
                    res["err"] = e

        th = threading.Thread(target=extender, daemon=True)
        th.start()
        seg.clear()
        so, t_smem, t_chain, kms = 0, 0.0, 0.0, 0.0
        try:
            for k in range(P):
                a, b = bounds[k], bounds[k + 1]
                t1 = time.perf_counter()
                bsw._check(fmi.collect_intv_device(d_reads.ptr, d_off.ptr + 8 * a, d_len.ptr + 4 * a, b - a, 150,
                                                   d_mems.ptr + a * cap * MZ, cap, d_cnt.ptr + 4 * a, mopt))
                kms += fmi.last_kernel_ms()
                t2 = time.perf_counter()
                rc, nk = fmi.mem_chain_device(d_len.ptr + 4 * a, b - a, d_mems.ptr + a * cap * MZ, cap,
                                              d_cnt.ptr + 4 * a, bufs["seeds"].ptr + so * SZ, bufs["sr"].ptr + 4 * so,
                                              bufs["sc"].ptr + 4 * so, sc_cap[0] - so, copt)
                if rc == -34:                            # sized by the sequential warm-up step: not expected
                    raise RuntimeError(f"pipelined step: batch {k} needs {nk} seed slots past {so} of {sc_cap[0]}")
                bsw._check(rc)
                t_smem += t2 - t1
                t_chain += time.perf_counter() - t2
                seg.append((a, so, nk))
                q.put((a, b, so, nk))
                so += nk
        finally:
            q.put(None)
            th.join()
        if res["err"] is not None:
            raise res["err"]
        smem_ms[0] = kms
        agg = bsw.ChainStats()
        for s in res["st"]:
            agg.rounds = max(agg.rounds, s.rounds)
            agg.n_extended += s.n_extended
            agg.n_skipped += s.n_skipped
            for j in range(4):
                agg.n_pairs[j] += s.n_pairs[j]
        return so, agg, (t_smem, t_chain, res["t"])

    if P > 1:
        step()                                           # sizes the seed buffers (grown here if short)
        log("sizing step done")
    for _ in range(args.warmup):
        step() if P == 1 else step_pipe()
        log("warm-up step done")
    barrier(world)
    t = time.perf_counter()
    n_ext, sts, parts = 0, [], []
    for _ in range(args.steps):
        ns, st, pt = step() if P == 1 else step_pipe()
        n_ext += sum(st.n_pairs)
        sts.append(st)
        parts.append(pt)
    barrier(world)
    dt = time.perf_counter() - t
    dt_max = allreduce_max(dt, world)
    n_ext_all = allreduce_sum(n_ext, world)
    seeds = bufs["seeds"].download(np.zeros(ns, dtype=bsw.SEED_DTYPE))
    sr = bufs["sr"].download(np.zeros(ns, dtype=np.int32))
    sc = bufs["sc"].download(np.zeros(ns, dtype=np.int32))
    out = bufs["out"].download(np.zeros(ns, dtype=bsw.ALNREG_DTYPE))
    ext = bufs["ext"].download(np.zeros(ns, dtype=np.int32))
    for a, so, nk in (seg if P > 1 else []):             # batch-relative read numbers -> the step's
        sr[so:so + nk] += a
    if args.dump:                                    # every rank: its shard's seeds and regions (tests)
        np.savez(f"{args.dump}.rank{rank}.npz", seeds=seeds, sr=sr, sc=sc, out=out, ext=ext)
    if rank != 0:
        return
    st = sts[-1]
    pm = np.mean(np.array(parts), axis=0) * 1e3
    reads_s = n * world * args.steps / dt_max / 1e6
    best = np.zeros(n, np.int32)
    np.maximum.at(best, sr[ext == 1], out["truesc"][ext == 1])
    value = reads_s if c1 else n_ext_all / dt_max / 1e6
    out_j = {
        "metric": "M reads/sec through GPU seeding + chaining + extension (C1)" if c1 else METRIC,
        "value": round(value, 3), "unit": "M reads/s" if c1 else UNIT, "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt_max / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16",
        "data": ("the reference's own C1 data (benchmark_threading.sh:42-70 generator, regenerated bit-exactly)"
                 if c1 else "synthetic PE reads (bench.pe_reads) from a bsw_synth.c random reference"),
        "config": {"workload": ("C1: 10K exact 150 bp SE reads vs the 1 Mb reference" if c1 else
                                f"C4 front end: {n} PE 150 bp reads/GPU vs a {args.ref_mb} Mb random reference") +
                               " -- FM-index SMEM seeding -> SA + mem_chain + mem_chain_flt -> mem_chain2aln, all on "
                               "the GPU, index / reads / two-strand text resident in HBM",
                   "reads_per_gpu": n, "ref_bases": int(len(ref)), "parallelism": f"shard{world} (independent reads)",
                   **({"seeding_options_EXPERIMENT": mo_kw} if mo_kw else {})},
        "reads_per_s_M": round(reads_s, 3),
        "extensions_per_s_M": round(n_ext_all / dt_max / 1e6, 3),
        "stage_ms": {"smem": round(float(pm[0]), 3), "chain": round(float(pm[1]), 3),
                     "chain2aln": round(float(pm[2]), 3),
                     **({"note": f"{P} batches: chain2aln of batch k on a second thread while batch k + 1 is "
                                 "seeded and chained -- the three stage times overlap"} if P > 1 else {})},
        "pipeline_batches": P,
        "smem_kernel_ms": round(smem_ms[0], 3),
        "seeds_per_read": round(ns / n, 3), "chains_per_read": round(float(len(np.unique(sr.astype(np.int64) * 65536 + sc))) / n, 3),
        "extended_fraction": round(st.n_extended / max(1, ns), 4), "rounds": st.rounds,
        "extensions_per_step_rank0": list(st.n_pairs),
        "full_length_fraction": round(float(np.mean(best == 150)), 4) if c1 else None,
        "index_build_s": round(build_s, 2), "synth_gen_s": round(gen_s, 2),
        "index": {"wide_64bit": bool(2 * len(ref) + 2 >= 2**32), "text_mode": not args.fmi_blocks_only,
                  "device_bytes": int(fmi.info().device_bytes),
                  "built_on": "gpu" if len(ref) >= (64 << 20) else "host"},
    }
    if world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # CPU baseline leg only (test infrastructure)
        nt = cpu_leg_threads()
        # the product's SA skips the oracle's comparison sort; past 512 Mb the oracle's LEAN form
        # (occurrence checkpoints every 64 rows + an SA sampled every 32 rows resolved by LF walks,
        # ~1.8 B per row) replaces its plain 42-B-per-row tables (~250 GB at 3 Gb)
        lean = len(ref) > 512_000_000
        S = min(n, (2_000 if lean else 10_000) * nt)
        t = time.perf_counter()
        sa_full = fmi.sa()
        fr = oracle.FmiRef(ref, sa=sa_full, lean=lean, nthreads=nt)
        del sa_full
        fsa = fr if lean else fr.sa()
        log(f"CPU leg: oracle index ({'lean' if lean else 'full'}) in {time.perf_counter() - t:.1f} s")

        def cpu_front(m, threads):
            mm, cn = fr.collect_intv(reads[:int(off[m - 1] + lens[m - 1])], off[:m], lens[:m], cap=cap,
                                     nthreads=threads)
            a, b, c = oracle.mem_chain(fsa, len(ref), lens[:m], mm, cn)
            return (a, b, c) + oracle.chain2aln(oracle.make_params(), opt, T, reads, off[:m], lens[:m], a, b, c,
                                                nthreads=threads)
        S1 = min(n, 2_000 if lean else 10_000)
        t = time.perf_counter()
        cpu_front(S1, 1)
        dt_1 = time.perf_counter() - t
        oracle.FmiRef.counters(reset=True)
        t = time.perf_counter()
        w_seeds, w_sr, w_sc, want, wext = cpu_front(S, nt)
        dt_cpu = time.perf_counter() - t
        n_bext, n_blocks = oracle.FmiRef.counters()
        k = int(np.searchsorted(sr, S))
        same = bool(len(w_seeds) == k and np.array_equal(w_sr, sr[:k]) and np.array_equal(w_sc, sc[:k]) and
                    np.array_equal(wext, ext[:k]) and all(np.array_equal(want[f], out[:k][f])
                                                          for f in bsw.ALNREG_DTYPE.names))
        rps = S / dt_cpu / 1e6
        out_j["cpu_baseline"] = {
            "value": round(rps, 5) if c1 else None, "unit": "M reads/s", "cores": nt, "kind": "oracle",
            "kind_note": "the scalar oracle pipeline (oracle/*.c restatements of bwa's algorithms, written for "
                         "checking, not speed) -- NOT the reference's optimized CPU path; see reference_published",
            "reads_per_s_M": round(rps, 5), "reads_per_s_M_1thread": round(S1 / dt_1 / 1e6, 5),
            "sample": f"first {S} reads; oracle/fmi_ref.c collect_intv + oracle/chain_ref.c mem_chain/mem_chain_flt + "
                      f"oracle/ext_ref.c chain2aln (scalar ksw_extend2) on {nt} threads (collect and chain2aln "
                      f"split by read; chaining 1 thread), index built from the product's suffix array, not timed"
                      + (" (lean oracle index: 64-row occurrence checkpoints, SA sampled every 32 rows + LF walks)"
                         if lean else ""),
            "host": host_cpu_info(),
            "outputs_identical_to_gpu": same,
        }
        rate = rps
        if not c1:
            n_cpu = int(np.sum(wext * ((w_seeds["qbeg"] > 0).astype(int) +
                                       ((w_seeds["qbeg"] + w_seeds["len"]) < lens[w_sr]).astype(int))))
            rate = n_cpu / dt_cpu / 1e6
            out_j["cpu_baseline"].update(value=round(rate, 5), unit=UNIT)
        out_j["cpu_baseline"].update(per_core_rate=round(rate / nt, 6), node_extrapolated=node_extrapolation(rate, nt))
        # the SMEM kernel's HBM roofline: algorithmic bytes = the reference algorithm's occurrence-
        # block loads (bwa-mem2 CP_OCC: one 64-B block per backward extension, two when the interval
        # spans blocks; counted by the oracle's walk on this sample) x 64 B per read, plus the read
        # bytes; achieved = those bytes for every read of the step / the SMEM kernel time of the step
        # (the GPU's k-mer table and text mode skip part of these loads: achieved may pass traffic)
        alg_per_read = n_blocks * 64.0 / S + float(np.mean(lens))
        smem_s = smem_ms[0] * 1e-3
        ach = alg_per_read * n / smem_s / 1e9
        out_j["roofline"] = smem_roofline(args, ach, {
            "kernel": "smem_kernel",
            "algorithmic": f"{alg_per_read:.0f} B per read ({n_blocks / S:.1f} occurrence-block loads x 64 B "
                           f"+ the read) x {n} reads per step", "launch_ms_per_step": round(smem_s * 1e3, 3),
            "backward_extensions_per_read": round(n_bext / S, 1)})
    if "roofline" not in out_j:
        # no CPU leg (--no-cpu, N > 1): the SMEM roofline from this workload's PMC pass alone
        out_j["roofline"] = smem_roofline(args, None, {
            "kernel": "smem_kernel", "launch_ms_per_step": round(smem_ms[0], 3),
            "algorithmic": "logical occurrence-block loads: counted by the CPU leg only"})
    if not c1:
        # the reference's own published bwa-mem2 rate (another machine and another dataset, SAM output
        # included): beside the oracle leg, never as the baseline of a ratio
        out_j["reference_published"] = {
            "value": 0.130378, "unit": "M reads/s", "threads": 16,
            "machine": "AWS Graviton4 c8g.4xlarge (16 vCPUs, Neoverse-V2)",
            "dataset": "human chr22 (~50 MB reference), 1M x 150 bp reads; bwa-mem2 mem end to end incl. SAM",
            "source": "/root/reference/GRAVITON4_BENCHMARK_RESULTS.md:21-30",
            "note": "another machine and another dataset: quoted for scale, not a measured ratio"}
    fmi.close()
    print(json.dumps(out_j), flush=True)


def main_mate(args, rank, local, world):
    """Mate-rescue batch (include/bsw_mate.h): per GPU `--jobs` ksw_align2 jobs as upstream's
    mem_sam_pe_batch builds them -- a 150 bp read vs a 550 bp window around the expected mate
    position (80% hold the mate), xtra = KSW_XSUBO | KSW_XSTART | KSW_XBYTE | 19 -- resident in
    HBM.  A step = one bsw_ksw_align2_device over the batch (bucketing, forward pass, reverse
    XSTART pass).  Work per job = the forward pass's full-width cells (ncol = slen*P columns x
    tlen rows, bsw_mate_stats_t.cells_fwd) plus the reverse pass."""
    t0 = time.perf_counter()
    ref = bsw.synth_reference(args.ref_mb * 1_000_000, seed=7)
    pairs, qer = bsw.synth_mates(ref, args.jobs, base=rank * args.jobs)
    gen_s = time.perf_counter() - t0
    d_pairs = hiprt.DeviceBuffer.from_array(pairs)
    d_ref = hiprt.DeviceBuffer.from_array(ref)
    d_qer = hiprt.DeviceBuffer.from_array(qer)
    aln = np.zeros(args.jobs, dtype=bsw.KSWR_DTYPE)
    d_aln = hiprt.DeviceBuffer.from_array(aln)
    eng = bsw.Engine(device=local)

    def step():
        bsw.ksw_align2_device(eng, d_pairs.ptr, d_ref.ptr, d_qer.ptr, args.jobs, d_aln.ptr)
        return bsw.mate_last_stats(eng)

    for _ in range(args.warmup):
        step()
    barrier(world)
    t = time.perf_counter()
    sts = [step() for _ in range(args.steps)]
    barrier(world)
    dt = time.perf_counter() - t
    dt_max = allreduce_max(dt, world)
    d_aln.download(aln)
    if rank != 0:
        return
    st = sts[-1]
    fwd_ms = float(np.mean([x.fwd_ms for x in sts]))
    rev_ms = float(np.mean([x.rev_ms for x in sts]))
    value = args.jobs * world * args.steps / dt_max / 1e6
    achieved = st.cells_fwd * OPS_PER_CELL / (fwd_ms * 1e-3) / 1e12
    out = {
        "metric": "M mate-rescue alignments/sec (150 bp read vs 550 bp window, ksw_align2)",
        "value": round(value, 3), "unit": "M alignments/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (bsw_synth.c mates, seed 42)",
        "config": {"workload": f"mate rescue: {args.jobs} jobs/GPU resident in HBM, 150 bp read vs 550 bp "
                               f"window of a {args.ref_mb} Mb random reference, KSW_XSUBO|XSTART|XBYTE",
                   "jobs_per_gpu": args.jobs, "parallelism": f"shard{world} (independent jobs)",
                   "n_fwd": st.n_fwd, "n_rev": st.n_rev},
        "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": round(VALU_PEAK_TOPS, 1),
                     "unit": "TOP/s", "frac": round(achieved / VALU_PEAK_TOPS, 4),
                     **traffic_for(args, "mate_kernel", prefix=True), "pmc_key": workload_key(args),
                     "kernel": "mate forward pass", "launch_ms": round(fwd_ms, 4),
                     "cells_per_s": round(st.cells_fwd / (fwd_ms * 1e-3) / 1e12, 4),
                     "algorithmic": f"{OPS_PER_CELL} int ops x {st.cells_fwd} forward cells per launch"},
        "rev_pass_ms": round(rev_ms, 4),
    }
    if world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # CPU baseline leg only (test infrastructure)
        cores = args.cpu_threads or len(os.sched_getaffinity(0))
        S = min(args.jobs, max(100_000, 2_000 * cores))
        mat = list(bsw.default_params().mat)
        t = time.perf_counter()
        want = oracle.ksw_align2_batch(pairs[:S], ref, qer, mat, nthreads=cores)
        dt_cpu = time.perf_counter() - t
        out["cpu_baseline"] = {
            "value": round(S / dt_cpu / 1e6, 4), "unit": "M alignments/s", "cores": cores, "kind": "port",
            "sample": f"first {S} jobs; oracle/ksw_align_ref.c (striped ksw_u8/ksw_i16 restated, scalar "
                      f"loops over the SIMD lanes), {cores} threads",
            "outputs_identical_to_gpu": bool(all(np.array_equal(want[f], aln[:S][f])
                                                 for f in bsw.KSWR_DTYPE.names)),
        }
    out["synth_gen_s"] = round(gen_s, 2)
    print(json.dumps(out), flush=True)


def main_global(args, rank, local, world):
    """Global alignment + CIGAR batch (include/bsw_global.h): per GPU `--jobs` ksw_global2 jobs as
    bwa_gen_cigar2 issues them for final alignments -- a 150 bp read vs exactly the reference span
    it covers (2% substitutions, 0.2% short indels), band w by bwa_gen_cigar2's rule (~35) --
    resident in HBM.  A step = one bsw_ksw_global2_device over the batch (plan, sort, banded DP
    with the traceback matrix in HBM, per-lane traceback, CIGARs written to HBM)."""
    t0 = time.perf_counter()
    ref = bsw.synth_reference(args.ref_mb * 1_000_000, seed=7)
    pairs, qer = bsw.synth_globals(ref, args.jobs, base=rank * args.jobs)
    gen_s = time.perf_counter() - t0
    stride = 64
    d_pairs = hiprt.DeviceBuffer.from_array(pairs)
    d_ref = hiprt.DeviceBuffer.from_array(ref)
    d_qer = hiprt.DeviceBuffer.from_array(qer)
    d_cig = hiprt.DeviceBuffer(args.jobs * stride * 4)
    d_nc = hiprt.DeviceBuffer(args.jobs * 4)
    eng = bsw.Engine(device=local)

    def step():
        bsw.ksw_global2_device(eng, d_pairs.ptr, d_ref.ptr, d_qer.ptr, args.jobs, d_cig.ptr, stride, d_nc.ptr)
        return bsw.global_last_stats(eng)

    for _ in range(args.warmup):
        step()
    barrier(world)
    t = time.perf_counter()
    sts = [step() for _ in range(args.steps)]
    barrier(world)
    dt = time.perf_counter() - t
    dt_max = allreduce_max(dt, world)
    res = np.empty_like(pairs)
    d_pairs.download(res)
    cig = np.empty((args.jobs, stride), dtype=np.uint32)
    d_cig.download(cig)
    nc = np.empty(args.jobs, dtype=np.int32)
    d_nc.download(nc)
    if rank != 0:
        return
    st = sts[-1]
    kms = float(np.mean([x.kernel_ms for x in sts]))
    value = args.jobs * world * args.steps / dt_max / 1e6
    bsw.ksw_global2_device(eng, d_pairs.ptr, d_ref.ptr, d_qer.ptr, args.jobs, 0, 0, 0)   # scores only
    so_ms = bsw.global_last_stats(eng).kernel_ms
    out = {
        "metric": "M global alignments with CIGAR/sec (150 bp read vs its reference span, ksw_global2)",
        "value": round(value, 3), "unit": "M alignments/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int16", "data": "synthetic (bsw_synth.c globals, seed 42)",
        "config": {"workload": f"global + CIGAR: {args.jobs} jobs/GPU resident in HBM, 150 bp read vs its "
                               f"reference span, w by bwa_gen_cigar2 (opt->w 100), CIGAR stride {stride}",
                   "jobs_per_gpu": args.jobs, "parallelism": f"shard{world} (independent jobs)",
                   "n_lane": st.n_lane, "n_wide": st.n_wide, "n_launches": st.n_launches,
                   "traceback_window": ("full band" if os.environ.get("BSW_GLOB_TB_DW") == "0" else
                                        f"narrow corridor, {os.environ.get('BSW_GLOB_TB_DW', '3')} dwords per row"),
                   "n_tb_retry": st.n_tb_retry, "z_bytes_per_step": st.z_bytes},
        "roofline": {"bound": "valu", "achieved": round(st.cells * OPS_PER_CELL / (kms * 1e-3) / 1e12, 3),
                     "peak": round(VALU_PEAK_TOPS, 1), "unit": "TOP/s",
                     "frac": round(st.cells * OPS_PER_CELL / (kms * 1e-3) / 1e12 / VALU_PEAK_TOPS, 4),
                     **traffic_for(args, "glob_lane_kernel", prefix=True), "pmc_key": workload_key(args),
                     "kernel": "glob_lane_kernel<160> (DP + traceback)", "launch_ms": round(kms, 4),
                     "cells_per_s": round(st.cells / (kms * 1e-3) / 1e12, 4),
                     "traceback_matrix_GBps": round(st.z_bytes / (kms * 1e-3) / 1e9, 1),
                     "algorithmic": f"{OPS_PER_CELL} int ops x {st.cells} band cells per step"},
        "cigar_ops_mean": round(float(np.mean(nc[nc > 0])), 3),
        "score_only_kernel_ms": round(so_ms, 4),
    }
    if world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # CPU baseline leg only (test infrastructure)
        cores = args.cpu_threads or len(os.sched_getaffinity(0))
        S = min(args.jobs, max(200_000, 4_000 * cores))
        mat = list(bsw.default_params().mat)
        t = time.perf_counter()
        ws, wc, wn = oracle.ksw_global2_batch(pairs[:S], ref, qer, mat, stride=stride, nthreads=cores)
        dt_cpu = time.perf_counter() - t
        same = bool(np.array_equal(ws, res["score"][:S]) and np.array_equal(wn, nc[:S]) and
                    all(np.array_equal(wc[i, :wn[i]], cig[i, :wn[i]]) for i in range(0, S, 97) if wn[i] > 0))
        out["cpu_baseline"] = {
            "value": round(S / dt_cpu / 1e6, 4), "unit": "M alignments/s", "cores": cores, "kind": "port",
            "sample": f"first {S} jobs; oracle/ksw_global_ref.c (scalar ksw_global2 restated, as bwa-mem2 "
                      f"runs it per alignment), {cores} threads",
            "outputs_identical_to_gpu": same,
        }
    out["synth_gen_s"] = round(gen_s, 2)
    print(json.dumps(out), flush=True)


HBM_PEAK_GBS = 8000.0              # MI355X HBM3E (MI355X_MICROARCH.md)


def smem_roofline(args, logical_gbps: float, extra: dict) -> dict:
    """The SMEM kernel's HBM roofline.  With a PMC pass of this workload: achieved / frac from the
    COUNTED HBM bytes per launch over the traced launch time (what the memory system moved); the
    logical rate -- every occurrence-block load the reference algorithm issues counted as 64 B of
    HBM traffic, although the L2 serves ~30% of them and the GPU's k-mer table / text mode skip
    others -- beside it as logical_GBps.  Without one: the logical rate, labelled as such."""
    t = traffic_for(args, "smem_kernel")
    r = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", **t, "pmc_key": workload_key(args),
         "logical_GBps": None if logical_gbps is None else round(logical_gbps, 1),
         "logical_frac": None if logical_gbps is None else round(logical_gbps / HBM_PEAK_GBS, 4)}
    if t.get("counter_GBps"):
        r.update(achieved=t["counter_GBps"], frac=round(t["counter_GBps"] / HBM_PEAK_GBS, 4),
                 basis="PMC-counted HBM bytes per launch / traced launch time (this workload's pass)")
    elif logical_gbps is None:          # (no CPU leg to count the logical loads, no PMC pass)
        r.update(achieved=None, frac=None, basis="no PMC pass of this workload and no CPU leg: unmeasured")
    else:
        r.update(achieved=round(logical_gbps, 1), frac=round(logical_gbps / HBM_PEAK_GBS, 4),
                 basis="logical occurrence-block loads x 64 B (no PMC pass of this workload)")
    r.update(extra)
    r["note"] = "serial chains of dependent loads: latency-bound, reported against the HBM roof"
    return r


def seeding_reference(n: int, seed: int = 7):
    """Random reference (codes 0..3) with ~10% interspersed repeat copies: segments of 300-5000
    bases copied elsewhere with 1% divergence, so seeds have multiple occurrences and the
    re-seeding / LAST-like passes fire as on a real genome."""
    rng = np.random.default_rng(seed)
    ref = rng.integers(0, 4, n, dtype=np.uint8)
    copied = 0
    while copied < n // 10:
        L = int(rng.integers(300, 5000))
        a, b = (int(x) for x in rng.integers(0, n - L, 2))
        seg = ref[a:a + L].copy()
        m = rng.random(L) < 0.01
        seg[m] = (seg[m] + rng.integers(1, 4, int(m.sum()))) % 4
        if rng.random() < 0.5:
            seg = (3 - seg[::-1]).astype(np.uint8)
        ref[b:b + L] = seg
        copied += L
    return ref


def seeding_reads(ref, n: int, L: int, seed: int):
    """n reads of L bases from either strand, 1% substitutions, 0.1% N, 5% random reads"""
    rng = np.random.default_rng(seed)
    pos = rng.integers(0, len(ref) - L, n)
    reads = ref[pos[:, None] + np.arange(L)[None, :]]
    rc = rng.random(n) < 0.5
    reads[rc] = (3 - reads[rc][:, ::-1]).astype(np.uint8)
    rnd = rng.random(n) < 0.05
    reads[rnd] = rng.integers(0, 4, (int(rnd.sum()), L), dtype=np.uint8)
    sub = rng.random((n, L)) < 0.01
    reads[sub] = ((reads[sub] + rng.integers(1, 4, int(sub.sum()))) % 4).astype(np.uint8)
    reads[rng.random((n, L)) < 0.001] = 4
    return np.ascontiguousarray(reads).reshape(-1), np.arange(n, dtype=np.int64) * L, np.full(n, L, np.int32)


def main_smem(args, rank, local, world):
    """FM-index SMEM seeding (include/bsw_fmi.h): per GPU `--reads` 151 bp
    reads resident in HBM against the FM-index of a `--ref-mb` reference (+ its reverse
    complement) resident in HBM.  A step = one bsw_mem_collect_intv_device over the batch
    (mem_collect_intv: SMEMs, re-seeding, LAST-like seeds, sorted).  Roofline: HBM bytes = the
    64-byte occurrence blocks the backward extensions touch (counted by the oracle on a sample)
    over the kernel time -- the walk is a chain of dependent loads, so this is a latency-bound
    kernel measured against the bandwidth roof."""
    L, cap = 151, 160
    t0 = time.perf_counter()
    ref = seeding_reference(args.smem_ref_mb * 1_000_000)
    reads, off, lens = seeding_reads(ref, args.reads, L, seed=11 + rank)
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    fmi = bsw.Fmi(ref, device=local, flags=(bsw.FMI_NO_TEXT if args.fmi_blocks_only else None))
    build_s = time.perf_counter() - t0
    d_reads, d_off, d_len = (hiprt.DeviceBuffer.from_array(a) for a in (reads, off, lens))
    d_mems = hiprt.DeviceBuffer(args.reads * cap * 32)
    d_cnt = hiprt.DeviceBuffer(args.reads * 4)

    def step():
        rc = fmi.collect_intv_device(d_reads.ptr, d_off.ptr, d_len.ptr, args.reads, L, d_mems.ptr, cap, d_cnt.ptr)
        if rc != 0:
            raise SystemExit(f"bsw_mem_collect_intv_device failed: {rc}")
        return fmi.last_kernel_ms()

    for _ in range(args.warmup):
        step()
    barrier(world)
    t = time.perf_counter()
    kms = [step() for _ in range(args.steps)]
    barrier(world)
    dt = time.perf_counter() - t
    dt_max = allreduce_max(dt, world)
    if rank != 0:
        return
    cnt = d_cnt.download(np.zeros(args.reads, dtype=np.int32))
    kernel_ms = float(np.median(kms))
    value = args.reads * world * args.steps / dt_max / 1e6
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # algorithmic-bytes count and the CPU baseline leg (test infrastructure)
    S = min(args.reads, 20_000)
    # the oracle's suffix array is a comparison sort: past 32 Mb it counts the blocks per read on a
    # 16 Mb reference of the same generator with reads of the same generator (a proxy, labelled)
    small = args.smem_ref_mb <= 32
    o_ref = ref if small else seeding_reference(16_000_000)
    o = oracle.FmiRef(o_ref)
    o_reads = reads if small else seeding_reads(o_ref, S, L, seed=11 + rank)[0]
    oracle.FmiRef.counters(reset=True)
    o_out, o_cnt = o.collect_intv(o_reads, off[:S], lens[:S], cap=cap, nthreads=1)
    n_ext, n_blk = oracle.FmiRef.counters(reset=True)
    bytes_per_read = n_blk * 64 / S
    achieved = bytes_per_read * args.reads / (kernel_ms * 1e-3) / 1e9
    out = {
        "metric": "M reads seeded/sec (151 bp, mem_collect_intv: SMEM + re-seeding + LAST-like passes)",
        "value": round(value, 3), "unit": "M reads/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32 (FM-index rows)", "data": "synthetic (seed 7 reference "
        "with 10% repeat copies; reads seed 11, 1% substitutions, 0.1% N, 5% random)",
        "config": {"workload": f"SMEM seeding: {args.reads} reads/GPU x {L} bp resident in HBM vs the FM-index of a "
                               f"{args.smem_ref_mb} Mb reference + reverse complement resident in HBM, bwa mem defaults "
                               f"(-k 19, split 1.5/10, max_mem_intv 20)",
                   "reads_per_gpu": args.reads, "parallelism": f"shard{world} (independent reads)",
                   "index_device_bytes": fmi.info().device_bytes, "index_build_s": round(build_s, 2),
                   "mems_per_read": round(float(cnt.mean()), 2)},
        "roofline": smem_roofline(args, achieved, {
            "kernel": "smem_kernel", "launch_ms": round(kernel_ms, 4),
            "algorithmic": f"{bytes_per_read:.0f} B per read = 64-B occurrence blocks touched by "
                           f"{n_ext / S:.1f} backward extensions per read (oracle count on {S} reads"
                           f"{'' if small else ' vs a 16 Mb reference of the same generator'}) x "
                           f"{args.reads} reads per launch"}),
    }
    gpu_out = d_mems.download(np.zeros((args.reads, cap), dtype=bsw.BWTINTV_DTYPE))
    agree = bool(np.array_equal(o_cnt, cnt[:S]) and all(np.array_equal(o_out[i, :o_cnt[i]], gpu_out[i, :o_cnt[i]])
                                                          for i in range(S))) if small else None
    if world == 1 and not args.no_cpu and small:
        host = host_cpu_info()
        q = host.get("cgroup_cpu_quota")
        cores = args.cpu_threads or int(min(len(os.sched_getaffinity(0)), math.ceil(q) if q else 1 << 30))
        S2 = min(args.reads, max(20_000, 4_000 * cores))
        t = time.perf_counter()
        o.collect_intv(reads, off[:S2], lens[:S2], cap=cap, nthreads=cores)
        dt_cpu = time.perf_counter() - t
        out["cpu_baseline"] = {
            "value": round(S2 / dt_cpu / 1e6, 4), "unit": "M reads/s", "cores": cores, "kind": "port",
            "sample": f"first {S2} reads; oracle/fmi_ref.c (bwt_smem1a / bwt_seed_strategy1 / mem_collect_intv "
                      f"restated over a prefix-count occurrence table), {cores} threads (affinity set capped "
                      f"at the cgroup quota)", "host": host}
    out["outputs_identical_to_oracle_sample"] = agree
    out["synth_gen_s"] = round(gen_s, 2)
    print(json.dumps(out), flush=True)


def allreduce_sum(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


if __name__ == "__main__":
    main()
