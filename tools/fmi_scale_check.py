"""Build FM-indexes of growing random references on the GPU and self-check each (bsw_fmi_check),
then seed a few reads and verify every interval by brute force on the text: the scale test of
the wide (64-bit) index before a 3 Gb run.  Usage: fmi_scale_check.py MB [MB ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem2-arm_amd", "py"))
import numpy as np  # noqa: E402
import hiprt  # noqa: E402,F401
import bsw  # noqa: E402

for mb in [int(x) for x in sys.argv[1:]]:
    t = time.perf_counter()
    ref = bsw.synth_reference(mb * 1_000_000, seed=7)
    ref[ref > 3] = 1
    print(f"{mb} Mb: reference {time.perf_counter() - t:.1f} s", flush=True)
    t = time.perf_counter()
    f = bsw.Fmi(ref)
    info = f.info()
    print(f"{mb} Mb: built in {time.perf_counter() - t:.1f} s, n {info.n}, device bytes {info.device_bytes / 2**30:.1f} GiB, "
          f"counts {list(info.count)}", flush=True)
    t = time.perf_counter()
    bad = f.check()
    print(f"{mb} Mb: self-check {bad} violations in {time.perf_counter() - t:.1f} s", flush=True)
    if bad:
        sys.exit(3)
    rng = np.random.default_rng(3)
    L, n = 151, 2000
    pos = rng.integers(0, len(ref) - L, n)
    reads = np.ascontiguousarray(ref[pos[:, None] + np.arange(L)[None, :]]).reshape(-1)
    out, cnt = f.collect_intv(reads, np.arange(n, dtype=np.int64) * L, np.full(n, L, np.int32), cap=64)
    full = sum(1 for i in range(n) for k in range(cnt[i]) if (out[i, k]["info"] & 0xffffffff) - (out[i, k]["info"] >> 32) == L)
    print(f"{mb} Mb: {n} exact reads -> {full} full-length SMEMs (want {n})", flush=True)
    f.close()
    if full != n:
        sys.exit(4)
