"""Replay .bswb batch files through the engine.

usage: python tools/bswb_replay.py FILE.bswb [FILE ...] [--oracle] [--repeat K]
For each file: run the recorded batch with its recorded scoring / band / cell_bits, report the
event-timed kernel rate, and compare per pair with the recorded outputs (when the file has
them) and, with --oracle, with the CPU oracle.  Exit status 1 on any difference.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "bwa-mem2-arm_amd", "py"), os.path.join(ROOT, "oracle")]
import bsw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args()
    bad_total = 0
    for path in a.files:
        h, pairs, ref, qer = bsw.read_batch(path)
        eng = bsw.Engine(h.params)
        got = pairs.copy()
        for _ in range(a.repeat):
            eng.get_scores(got, ref, qer, h.w, h.cell_bits)
        st = eng.last_stats()
        rate = len(pairs) / (st.kernel_ms * 1e-3) / 1e6 if st.kernel_ms > 0 else float("nan")
        msg = f"{os.path.basename(path)}: {len(pairs)} pairs w={h.w} cell_bits={h.cell_bits} kernel {st.kernel_ms:.3f} ms ({rate:.1f} M pairs/s)"
        if h.flags & 1:
            bad = sum(int(np.sum(pairs[f] != got[f])) for f in bsw.OUT_FIELDS)
            msg += f", vs recorded outputs: {bad} field differences"
            bad_total += bad
        if a.oracle:
            import oracle
            want = pairs.copy()
            p = oracle.make_params(o_del=h.params.o_del, e_del=h.params.e_del, o_ins=h.params.o_ins,
                                   e_ins=h.params.e_ins, zdrop=h.params.zdrop, end_bonus=h.params.end_bonus,
                                   mat=list(h.params.mat))
            oracle.get_scores(p, want, ref, qer, h.w, nthreads=16)
            bad = sum(int(np.sum(want[f] != got[f])) for f in bsw.OUT_FIELDS)
            msg += f", vs oracle: {bad} field differences"
            bad_total += bad
        print(msg, flush=True)
        eng.close()
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
