#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/golden_v1.npz + manifest.json).

The reference (/root/reference) holds no fixtures, golden vectors or tests for this path
(SURVEY.md §4, §8c), so the golden outputs are produced by this repo's CPU oracle
(oracle/ksw_ext_ref.c = ksw_extend2 restated from SURVEY.md Appendix A), after it has
been cross-checked against the independent Python transcription (oracle/ksw_ext_ref.py)
and the hand-derived known answers in tests/test_oracle.py.  PARITY UNPINNED by the
reference itself; these fixtures pin the oracle against regressions and give the GPU
tests inputs whose expected outputs are fixed in the repository.

Batches (each with its own band w and scoring):
  b0  mixed random shapes (len 0..170 / 0..320), w=100      -- stale-column + wide routing
  b1  same generator, w=5  (narrow band; stale-column rule A.7 fires at small w)
  b2  same generator, w=1
  b3  C2-shaped (150/300, h0 in [19,100]), w=100
  b4  edge cases (lengths 0/1/2/15/16/17/.../160, all-N, repeats, h0 extremes), w=100
  b5  mixed shapes with non-default scoring (-A2 -B3 -O5,7 -E2,1 -d50 -L3), w=40
  b6  partial batches of 1, 15, 31, 32, 33, 50, 64, 100 pairs (the reference's planned
      SVE2 validation sizes, PHASE2_IMPLEMENTATION_SUMMARY.md:194-201), w=100
"""

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import bswgen  # noqa: E402
import oracle  # noqa: E402
from ksw_ext_ref import bwa_fill_scmat  # noqa: E402

DEFAULT = dict(o_del=6, e_del=1, o_ins=6, e_ins=1, zdrop=100, end_bonus=5, a=1, b=4)
ALT = dict(o_del=5, e_del=2, o_ins=7, e_ins=1, zdrop=50, end_bonus=3, a=2, b=3)


def batches():
    out = []
    out.append(("b0", bswgen.random_pairs(600, seed=101), 100, DEFAULT))
    out.append(("b1", bswgen.random_pairs(500, seed=102, tlen=(0, 200), qlen=(0, 120)), 5, DEFAULT))
    out.append(("b2", bswgen.random_pairs(400, seed=103, tlen=(0, 120), qlen=(0, 80)), 1, DEFAULT))
    out.append(("b3", bswgen.c2_like(400, seed=104), 100, DEFAULT))
    out.append(("b4", bswgen.edge_pairs(seed=105), 100, DEFAULT))
    out.append(("b5", bswgen.random_pairs(400, seed=106, tlen=(0, 250), qlen=(0, 160)), 40, ALT))
    for k, m in enumerate((1, 15, 31, 32, 33, 50, 64, 100)):
        out.append((f"b6_{m}", bswgen.random_pairs(m, seed=200 + k, tlen=(50, 300), qlen=(30, 150)), 100, DEFAULT))
    return out


def params_of(d):
    return oracle.make_params(o_del=d["o_del"], e_del=d["e_del"], o_ins=d["o_ins"], e_ins=d["e_ins"],
                              zdrop=d["zdrop"], end_bonus=d["end_bonus"],
                              mat=bwa_fill_scmat(d["a"], d["b"]))


def main():
    arrays = {}
    meta = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/ksw_ext_ref.c",
            "parity": "unpinned by the reference (no reference fixtures exist); oracle-generated",
            "batches": []}
    for name, (pairs, ref, qer), w, sc in batches():
        p = pairs.copy()
        oracle.get_scores(params_of(sc), p, ref, qer, w)
        arrays[f"{name}_pairs"] = p.view(np.int32).reshape(len(p), 14)
        arrays[f"{name}_ref"] = ref
        arrays[f"{name}_qer"] = qer
        meta["batches"].append({"name": name, "n": int(len(p)), "w": w, "scoring": sc})
    path = os.path.join(HERE, "golden_v1.npz")
    np.savez_compressed(path, **arrays)
    meta["sha256"] = hashlib.sha256(open(path, "rb").read()).hexdigest()
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    print(f"wrote {path} ({os.path.getsize(path)} B), {sum(b['n'] for b in meta['batches'])} pairs")


if __name__ == "__main__":
    main()
