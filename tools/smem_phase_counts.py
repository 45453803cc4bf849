"""Where the SMEM walk's occurrence-block loads go, per seeding phase (CPU, the oracle's
counters): pass-1 forward / backward sweep, pass-2 (re-seeding) forward / backward, pass 3.
Counts the extensions of intervals with s >= 2 (the GPU kernel serves s = 1 from the text) on a
random reference with bench.py's C4 reads (1% substitutions, 0.1% N).  With "repeats" the
reference is bench.seeding_reference (C4's: 10% interspersed copies at 1% divergence).  Also the
s = 2 extensions and how many of them keep s = 2 (the case a two-position text mode would serve).
  python tools/smem_phase_counts.py [ref_mb] [reads] [repeats]"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import oracle  # noqa: E402
import bench  # noqa: E402


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 16
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    rep = len(sys.argv) > 3 and sys.argv[3] == "repeats"
    ref = bench.seeding_reference(int(mb * 1e6)) if rep else np.random.default_rng(7).integers(0, 4, int(mb * 1e6), dtype=np.uint8)
    t0 = time.time()
    f = oracle.FmiRef(ref)
    print(f"index {mb} Mb built in {time.time() - t0:.1f} s", flush=True)
    reads, off, lens = bench.pe_reads(ref, nr // 2)
    L = oracle.lib()
    L.oracle_fmi_phase_counters.argtypes = [ctypes.c_void_p, ctypes.c_int]
    c = np.zeros(15, dtype=np.uint64)
    L.oracle_fmi_s2_counters.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    s2 = np.zeros(15, dtype=np.uint64)
    kt = max(0, min(15, int(np.floor(np.log(2 * len(ref)) / np.log(4))) - 1))   # the GPU's table depth
    L.oracle_fmi_phase_counters(c.ctypes.data, 1)
    L.oracle_fmi_s2_counters(s2.ctypes.data, 1, kt)
    iv, cnt = f.collect_intv(reads, off, lens, nthreads=8)
    L.oracle_fmi_phase_counters(c.ctypes.data, 0)
    L.oracle_fmi_s2_counters(s2.ctypes.data, 0, kt)
    s2 = s2.reshape(5, 3) / len(lens)
    c = c.reshape(5, 3) / len(lens)
    names = ["pass1 forward", "pass1 backward", "pass2 forward", "pass2 backward", "pass3"]
    tot = c[:, 1].sum()
    print(f"reference {'with 10% repeat copies' if rep else 'random'}; table depth kt = {kt}")
    print(f"per read ({len(lens)} reads, {cnt.mean():.2f} intervals/read): extensions, s>=2 extensions (share), "
          f"s>=2 block loads | block walks past the table: all, at s = 2, s = 2 kept")
    for n, r, t in zip(names, c, s2):
        print(f"  {n:15s} {r[0]:8.1f} {r[1]:8.1f} ({100 * r[1] / tot:5.1f}%) {r[2]:8.1f} | {t[0]:8.1f} {t[1]:8.1f} {t[2]:8.1f}")
    print(f"  {'total':15s} {c[:, 0].sum():8.1f} {tot:8.1f}          {c[:, 2].sum():8.1f} | {s2[:, 0].sum():8.1f} "
          f"{s2[:, 1].sum():8.1f} {s2[:, 2].sum():8.1f}")


if __name__ == "__main__":
    main()
