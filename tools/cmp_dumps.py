"""Compare two bench.py --dump outputs (<a>.rank0.npz vs <b>.rank0.npz): every array equal.
Used to check that a pipelined c4mem step (--pipeline P) writes exactly what the sequential step
writes.  python tools/cmp_dumps.py <dump-a> <dump-b>"""
import sys

import numpy as np

a, b = (np.load(f"{p}.rank0.npz") for p in sys.argv[1:3])
bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
print({k: int(a[k].shape[0]) for k in a.files}, "identical" if not bad else f"DIFFER in {bad}")
sys.exit(1 if bad else 0)
