#!/usr/bin/env python3
"""Oracle cross-check at scale (test infrastructure; run by hand, output committed).

SURVEY.md §8(c) asks for the C restatement of ksw_extend2 (oracle/ksw_ext_ref.c) to equal an
independent transcription on >= 10^6 pairs of C2 shape.  The pure-Python transcription
(oracle/ksw_ext_ref.py) is far too slow for that, so the independent side here is the
vectorised numpy transcription (oracle/ksw_ext_np.py: numpy lanes in lock-step, every
Appendix A rule literal per lane), run in worker processes over chunks of the batch.

Workloads:
  C2     the bench batch itself (bsw_synth.c, seed 42): 1,000,000 pairs, 150/300, w = 100
  extra  100,000 pairs each of classes C2 does not reach: z-drop off, w = 200 with 200 bp
         queries, asymmetric gaps (e_del != e_ins, o_del != o_ins), tandem repeats (ties)

usage: python tests/oracle_crosscheck.py [--pairs 1000000] [--extra 100000] [--procs 8]
       [--out tests/golden/crosscheck_1e6.json]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "bwa-mem2-arm_amd", "py")]

import numpy as np  # noqa: E402

import bswgen  # noqa: E402
import oracle  # noqa: E402
from ksw_ext_np import ksw_extend2_lanes  # noqa: E402
from ksw_ext_ref import bwa_fill_scmat  # noqa: E402

FIELDS = ("score", "tle", "gtle", "qle", "gscore", "max_off")


def _np_chunk(args):
    pairs, ref, qer, sc, w = args
    return ksw_extend2_lanes(pairs, ref, qer, bwa_fill_scmat(sc["a"], sc["b"]), sc["o_del"], sc["e_del"],
                             sc["o_ins"], sc["e_ins"], w, sc["end_bonus"], sc["zdrop"])


def run(name, pairs, ref, qer, sc, w, procs, chunk=20_000):
    t0 = time.time()
    want = pairs.copy()
    oracle.get_scores(oracle.make_params(o_del=sc["o_del"], e_del=sc["e_del"], o_ins=sc["o_ins"], e_ins=sc["e_ins"],
                                         zdrop=sc["zdrop"], end_bonus=sc["end_bonus"],
                                         mat=bwa_fill_scmat(sc["a"], sc["b"])),
                      want, ref, qer, w, nthreads=procs)
    t_c = time.time() - t0
    t0 = time.time()
    jobs = [(pairs[a:a + chunk], ref, qer, sc, w) for a in range(0, len(pairs), chunk)]
    got = {f: [] for f in FIELDS}
    with ProcessPoolExecutor(max_workers=procs) as ex:
        for r in ex.map(_np_chunk, jobs):
            for f in FIELDS:
                got[f].append(r[f])
    t_np = time.time() - t0
    bad = np.zeros(len(pairs), bool)
    per_field = {}
    for f in FIELDS:
        g = np.concatenate(got[f]) if got[f] else np.zeros(0, np.int32)
        d = g != want[f]
        per_field[f] = int(d.sum())
        bad |= d
    res = {"workload": name, "pairs": int(len(pairs)), "w": w, "scoring": sc,
           "mismatched_pairs": int(bad.sum()), "mismatches_per_field": per_field,
           "c_oracle_s": round(t_c, 1), "numpy_lanes_s": round(t_np, 1),
           "output_checksum": int(np.bitwise_xor.reduce(
               (want["score"].astype(np.int64) * 1000003 + want["tle"] * 10007 + want["gtle"] * 101 +
                want["qle"] * 7 + want["gscore"] * 3 + want["max_off"]).astype(np.int64)))}
    print(json.dumps(res), flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--extra", type=int, default=100_000)
    ap.add_argument("--procs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "crosscheck_1e6.json"))
    args = ap.parse_args()
    import bsw
    default = dict(o_del=6, e_del=1, o_ins=6, e_ins=1, zdrop=100, end_bonus=5, a=1, b=4)
    out = {"what": "oracle/ksw_ext_ref.c (C, literal) vs oracle/ksw_ext_np.py (numpy lanes, independent "
                   "transcription of SURVEY.md Appendix A); parity of the oracle itself, unpinned by the reference",
           "script": "tests/oracle_crosscheck.py", "runs": []}
    pairs, ref, qer = bsw.synth_batch(args.pairs)
    out["runs"].append(run("C2 (bsw_synth.c seed 42, 150/300)", pairs, ref, qer, default, 100, args.procs))
    n = args.extra
    extra = [
        ("zdrop=0, C2-like", bswgen.c2_like(n, seed=11), dict(default, zdrop=0), 100),
        ("w=200, 200 bp query / 420 bp ref", bswgen.c2_like(n, seed=12, tlen=420, qlen=200, h0=(19, 120)), default, 200),
        ("asymmetric gaps -O6,4 -E1,3, mixed shapes", bswgen.random_pairs(n, seed=13),
         dict(o_del=6, e_del=1, o_ins=4, e_ins=3, zdrop=100, end_bonus=5, a=1, b=4), 100),
        ("tandem repeats (ties)", bswgen.repeat_pairs(n, seed=14), default, 100),
    ]
    for name, (p, r, q), sc, w in extra:
        out["runs"].append(run(name, p, r, q, sc, w, args.procs))
    out["total_pairs"] = sum(r["pairs"] for r in out["runs"])
    out["total_mismatched_pairs"] = sum(r["mismatched_pairs"] for r in out["runs"])
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"wrote {args.out}: {out['total_pairs']} pairs, {out['total_mismatched_pairs']} mismatched")
    return 1 if out["total_mismatched_pairs"] else 0


if __name__ == "__main__":
    sys.exit(main())
