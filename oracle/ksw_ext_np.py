"""CPU ORACLE, vectorised numpy transcription (test infrastructure only; never shipped).

A third, independent restatement of `ksw_extend2` (upstream bwa-mem2 v2.2.1 `src/ksw.cpp`
= lh3/bwa ksw.c) written from SURVEY.md Appendix A (A.1-A.7).  It runs MANY pairs in
lock-step, one numpy lane per pair -- the shape of the reference's own SIMD batch kernels
(`smithWaterman128_16`) -- while keeping every rule literal per lane:
the persistent per-pair `eh` row with its stale columns (A.7), the narrowing scans on both
band edges, the strict `m > max` update, the last-index tie rule, the z-drop test and the
per-lane break.  It shares no code with oracle/ksw_ext_ref.c or oracle/ksw_ext_ref.py; the
three must agree (tests/test_oracle.py, tests/oracle_crosscheck.py at 10^6 pairs).

PARITY UNPINNED by the reference: /root/reference holds no source, fixtures or tests for
this path; see oracle/ksw_ext_ref.c's header.
"""

from __future__ import annotations

import numpy as np

OUT = ("score", "tle", "gtle", "qle", "gscore", "max_off")


def _band_cap(qlen, w, maxsc, end_bonus, o, e):
    # A.2: (int)((double)(qlen * maxsc + end_bonus - o) / e + 1.0), at least 1 -- C truncation
    v = np.trunc((qlen.astype(np.float64) * maxsc + end_bonus - o) / e + 1.0).astype(np.int64)
    return np.minimum(w, np.maximum(v, 1))


def ksw_extend2_lanes(pairs, ref, qer, mat, o_del, e_del, o_ins, e_ins, w, end_bonus, zdrop):
    """Outputs for every SeqPair record in `pairs` (numpy structured array with the SeqPair
    fields): dict field -> int32 array.  ref / qer are the 1-byte code buffers (idr / idq)."""
    n = len(pairs)
    qlen = pairs["len2"].astype(np.int64)
    tlen = pairs["len1"].astype(np.int64)
    h0 = pairs["h0"].astype(np.int64)
    idr = pairs["idr"].astype(np.int64)
    idq = pairs["idq"].astype(np.int64)
    mat = np.asarray(mat, dtype=np.int64).reshape(5, 5)
    oe_del, oe_ins = o_del + e_del, o_ins + e_ins
    qmax = int(qlen.max()) if n else 0
    lanes = np.arange(n)
    # query codes per lane, padded (columns >= qlen are never in band)
    cols = np.arange(qmax + 2)
    qc = np.zeros((n, qmax + 2), dtype=np.int64)
    inq = cols[None, :] < qlen[:, None]
    qc[inq] = qer[(idq[:, None] + cols[None, :])[inq]]
    # A.1 row buffer: H[j] = eh[j].h, E[j] = eh[j].e for j in 0..qlen (+1 guard column)
    H = np.zeros((n, qmax + 2), dtype=np.int64)
    E = np.zeros((n, qmax + 2), dtype=np.int64)
    H[:, 0] = h0
    H[:, 1] = np.maximum(h0 - oe_ins, 0)
    # eh[j].h = eh[j-1].h - e_ins while eh[j-1].h > e_ins, for j = 2..qlen
    run = np.ones(n, dtype=bool)
    for j in range(2, qmax + 1):
        run &= (j <= qlen) & (H[:, j - 1] > e_ins)
        if not run.any():
            break
        H[run, j] = H[run, j - 1] - e_ins
    maxsc = max(0, int(mat.max()))
    wl = _band_cap(qlen, w, maxsc, end_bonus, o_ins, e_ins)
    wl = _band_cap(qlen, wl, maxsc, end_bonus, o_del, e_del)
    # A.3 state
    best, best_i, best_j = h0.copy(), np.full(n, -1, np.int64), np.full(n, -1, np.int64)
    max_ie, gscore, max_off = np.full(n, -1, np.int64), np.full(n, -1, np.int64), np.zeros(n, np.int64)
    beg, end = np.zeros(n, np.int64), qlen.copy()
    alive = np.ones(n, dtype=bool)
    tmax = int(tlen.max()) if n else 0
    for i in range(tmax):
        act = alive & (i < tlen)
        if not act.any():
            break
        # A.4 row setup
        beg = np.where(act, np.maximum(beg, i - wl), beg)
        end = np.where(act, np.minimum(np.minimum(end, i + wl + 1), qlen), end)
        t_i = np.zeros(n, np.int64)
        ta = act & (i < tlen)
        t_i[ta] = ref[idr[ta] + i]
        srow = mat[t_i]                                   # (n, 5): S(i, q) by query code
        h1 = np.where(beg == 0, np.maximum(h0 - (o_del + e_del * (i + 1)), 0), 0)
        f = np.zeros(n, np.int64)
        m = np.zeros(n, np.int64)
        mj = np.full(n, -1, np.int64)
        jlo = int(beg[act].min())
        jhi = int(end[act].max())
        for j in range(jlo, jhi):
            inb = act & (beg <= j) & (j < end)
            if not inb.any():
                continue
            Mv = H[:, j].copy()
            ev = E[:, j]
            H[inb, j] = h1[inb]
            S = srow[lanes, qc[:, j]]
            Mv = np.where(Mv != 0, Mv + S, 0)
            h = np.maximum(np.maximum(Mv, ev), f)
            h1 = np.where(inb, h, h1)
            mj = np.where(inb & ~(m > h), j, mj)
            m = np.where(inb, np.maximum(m, h), m)
            t = np.maximum(Mv - oe_del, 0)
            enew = np.maximum(ev - e_del, t)
            E[inb, j] = enew[inb]
            t = np.maximum(Mv - oe_ins, 0)
            f = np.where(inb, np.maximum(f - e_ins, t), f)
        # end of row
        ia = lanes[act]
        H[ia, end[act]] = h1[act]
        E[ia, end[act]] = 0
        jx = np.where(beg < end, end, beg)
        g = act & (jx == qlen)
        max_ie = np.where(g & ~(gscore > h1), i, max_ie)
        gscore = np.where(g, np.maximum(gscore, h1), gscore)
        brk = act & (m == 0)
        upd = act & ~brk & (m > best)
        best = np.where(upd, m, best)
        best_i = np.where(upd, i, best_i)
        best_j = np.where(upd, mj, best_j)
        max_off = np.where(upd, np.maximum(max_off, np.abs(mj - i)), max_off)
        if zdrop > 0:
            zc = act & ~brk & ~upd
            di, dj = i - best_i, mj - best_j
            dz = np.where(di > dj, best - m - (di - dj) * e_del, best - m - (dj - di) * e_ins)
            brk |= zc & (dz > zdrop)
        alive = alive & ~brk
        live = act & ~brk
        if not live.any():
            continue
        # narrowing: first nonzero eh in [beg, end) -> beg; last nonzero eh in [beg, end] -> end
        nz = (H != 0) | (E != 0)
        c = cols[None, :]
        lo = np.where(nz & (c >= beg[:, None]) & (c < end[:, None]), c, qmax + 5).min(axis=1)
        newbeg = np.minimum(lo, end)                      # none found: j stops at end
        hi = np.where(nz & (c >= newbeg[:, None]) & (c <= end[:, None]), c, -1).max(axis=1)
        hi = np.where(hi < newbeg, newbeg - 1, hi)        # none found: j stops at beg - 1
        beg = np.where(live, newbeg, beg)
        end = np.where(live, np.minimum(hi + 2, qlen), end)
    return {"score": best.astype(np.int32), "tle": (best_i + 1).astype(np.int32),
            "gtle": (max_ie + 1).astype(np.int32), "qle": (best_j + 1).astype(np.int32),
            "gscore": gscore.astype(np.int32), "max_off": max_off.astype(np.int32)}
