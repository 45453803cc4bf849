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

`python make_golden.py v2` writes golden_v2.npz + manifest_v2.json (round 2: the SURVEY.md
§8(c) classes v1 lacked -- z-drop off, w = 200, asymmetric gaps, ties):
  z0_c2 / z0_rand / z0_w5   zdrop = 0 (the `else if (zdrop > 0)` branch never breaks)
  w200_c2 / w200_long       w = 200 (band wider than the query; 200 bp queries -> wide kernel)
  asym_ins / asym_del       e_del != e_ins and o_del != o_ins (the non-packed lane kernel)
  ties                      tandem repeats: equal-score paths, last-index tie rules
v1 is left as generated in round 1.
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


ZDROP0 = dict(DEFAULT, zdrop=0)
ASYM_INS = dict(o_del=6, e_del=1, o_ins=4, e_ins=3, zdrop=100, end_bonus=5, a=1, b=4)
ASYM_DEL = dict(o_del=3, e_del=3, o_ins=8, e_ins=1, zdrop=80, end_bonus=5, a=1, b=4)


def batches_v2():
    return [
        ("z0_c2", bswgen.c2_like(400, seed=301), 100, ZDROP0),
        ("z0_rand", bswgen.random_pairs(400, seed=302), 100, ZDROP0),
        ("z0_w5", bswgen.random_pairs(300, seed=303, tlen=(0, 200), qlen=(0, 120)), 5, ZDROP0),
        ("w200_c2", bswgen.c2_like(300, seed=304), 200, DEFAULT),
        ("w200_long", bswgen.c2_like(200, seed=305, tlen=420, qlen=200, h0=(19, 120)), 200, DEFAULT),
        ("asym_ins", bswgen.random_pairs(400, seed=306, tlen=(0, 300), qlen=(0, 160)), 100, ASYM_INS),
        ("asym_del", bswgen.c2_like(300, seed=307), 50, ASYM_DEL),
        ("ties", bswgen.repeat_pairs(400, seed=308), 100, DEFAULT),
    ]


def params_of(d):
    return oracle.make_params(o_del=d["o_del"], e_del=d["e_del"], o_ins=d["o_ins"], e_ins=d["e_ins"],
                              zdrop=d["zdrop"], end_bonus=d["end_bonus"],
                              mat=bwa_fill_scmat(d["a"], d["b"]))


def main(version="v1"):
    arrays = {}
    meta = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/ksw_ext_ref.c",
            "parity": "unpinned by the reference (no reference fixtures exist); oracle-generated",
            "batches": []}
    for name, (pairs, ref, qer), w, sc in (batches() if version == "v1" else batches_v2()):
        p = pairs.copy()
        oracle.get_scores(params_of(sc), p, ref, qer, w)
        arrays[f"{name}_pairs"] = p.view(np.int32).reshape(len(p), 14)
        arrays[f"{name}_ref"] = ref
        arrays[f"{name}_qer"] = qer
        meta["batches"].append({"name": name, "n": int(len(p)), "w": w, "scoring": sc})
    path = os.path.join(HERE, f"golden_{version}.npz")
    np.savez_compressed(path, **arrays)
    meta["sha256"] = hashlib.sha256(open(path, "rb").read()).hexdigest()
    meta["file"] = os.path.basename(path)
    mname = "manifest.json" if version == "v1" else f"manifest_{version}.json"
    with open(os.path.join(HERE, mname), "w") as fh:
        json.dump(meta, fh, indent=1)
    print(f"wrote {path} ({os.path.getsize(path)} B), {sum(b['n'] for b in meta['batches'])} pairs")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "v1")
