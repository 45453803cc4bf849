"""Per-wave schedule of one pc_kernel launch on the C2 batch (experiment; GPU box):
   BSW_HIP_LIB=bwa-mem2-arm_amd/lib/libbsw_hip_stats.so python tools/pc_times.py [out.npz]
The stats build records, per wave, its start / end (s_memrealtime, 100 MHz), XCC id, HW_ID and
rows.  Printed: launch span, busy fraction of the wave slots (2 per SIMD x 4 SIMDs x 256 CUs),
ramp-up (first start -> all slots busy), tail (last time all slots were busy -> last end),
lifetime by position in the dispatch order (deciles), and what a longest-first order of the
same waves would give under a greedy list schedule (a simulation, not a measurement)."""
import ctypes
import heapq
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import numpy as np  # noqa: E402
import hiprt  # noqa: E402
import bsw  # noqa: E402

SLOTS = 2 * 4 * 256
TICK_US = 0.01                                  # s_memrealtime: 100 MHz


def greedy(dur, slots):
    """list schedule of `dur` in the given order on `slots` identical slots: makespan"""
    h = [0.0] * slots
    heapq.heapify(h)
    for d in dur:
        t = heapq.heappop(h)
        heapq.heappush(h, t + d)
    return max(h)


def main():
    n = int(os.environ.get("PAIRS", "1000000"))
    pairs, ref, qer = bsw.synth_batch(n)
    d = [hiprt.DeviceBuffer.from_array(a) for a in (pairs, ref, qer)]
    eng = bsw.Engine()
    L = bsw.hip_lib()
    L.bsw_pc_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(3):
        eng.get_scores_device(d[0].ptr, d[1].ptr, d[2].ptr, n, 100, 16)
    kms = eng.last_stats().kernel_ms
    nw = (n + 63) // 64
    buf = np.zeros((nw, 4), dtype=np.uint64)
    got = L.bsw_pc_times(buf.ctypes.data, nw)
    assert got == nw, got
    t0 = buf[:, 0].astype(np.int64)
    t1 = buf[:, 1].astype(np.int64)
    base = t0.min()
    s = (t0 - base) * TICK_US
    e = (t1 - base) * TICK_US
    life = e - s
    span = e.max()
    busy = life.sum() / (SLOTS * span)
    # occupancy over time
    ev = np.concatenate([np.stack([s, np.ones(nw)], 1), np.stack([e, -np.ones(nw)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    occ = np.cumsum(ev[:, 1])
    full = ev[occ >= SLOTS * 0.98, 0]
    ramp = full.min() if len(full) else float("nan")
    tail_from = full.max() if len(full) else float("nan")
    print(f"launch: {nw} waves, kernel_ms {kms:.3f}, span {span / 1e3:.3f} ms, busy fraction {busy:.3f}")
    print(f"ramp-up to 98% of {SLOTS} slots: {ramp:.1f} us; tail (below 98% until the end): {span - tail_from:.1f} us")
    print(f"max concurrent waves {int(occ.max())}")
    dec = np.array_split(np.arange(nw), 10)
    print("lifetime by dispatch-order decile (us, mean / p90): " +
          "  ".join(f"{life[i].mean():.0f}/{np.percentile(life[i], 90):.0f}" for i in dec))
    rows = buf[:, 3].astype(np.int64)
    print(f"rows per wave mean {rows.mean():.1f}; us per row {np.sum(life) / max(1, rows.sum()):.3f}")
    xcc = (buf[:, 2] >> np.uint64(32)).astype(np.int64)
    print("waves per XCC " + " ".join(str(int((xcc == k).sum())) for k in range(8)))
    mk_disp = greedy(life, SLOTS)
    mk_lpt = greedy(np.sort(life)[::-1], SLOTS)
    print(f"greedy list schedule of these lifetimes: dispatch order {mk_disp / 1e3:.3f} ms, "
          f"longest-first {mk_lpt / 1e3:.3f} ms, lower bound {life.sum() / SLOTS / 1e3:.3f} ms")
    if len(sys.argv) > 1:
        np.savez_compressed(sys.argv[1], times=buf)


if __name__ == "__main__":
    main()
