"""Independent, non-striped formulation of upstream ksw_u8 / ksw_i16 / ksw_align2 (mate-rescue
local Smith-Waterman) -- TEST INFRASTRUCTURE.

oracle/ksw_align_ref.c restates the SSE2 kernels literally (striped lanes, lazy-F loop with
its early exit).  This module derives the same results in plain query order, which is also
the formulation the GPU kernel implements:

  per row i, columns j = 0 .. ncol-1 (ncol = slen * P, positions >= qlen score 0):
    segment starts are j = k * slen; entering one, the in-segment F chain is reset to 0 and
    its outgoing value joins the cross-segment chain fx (what the lazy-F loop carries);
    H1 = max(Hdiag + S, E, f)            (u8: biased add, capped at 255, floored at 0)
    H  = max(H1, fx)                      (what the next row sees; fx decays by e_ins)
    E' = max(E - e_del, H1 - oe_del, 0)   (from H1: upstream does not redo E after lazy-F)
    f' = max(f - e_ins, H1 - oe_ins, 0)
    imax = max H1 over the row (upstream's row maximum is taken before lazy-F)
Agreement of the two on random inputs pins both."""

from __future__ import annotations

KSW_XBYTE, KSW_XSTOP, KSW_XSUBO, KSW_XSTART = 0x10000, 0x20000, 0x40000, 0x80000


def _shift(mat):
    mn = min(min(mat), 127)
    return (256 - (mn & 0xFF)) & 0xFF


def ksw_local(query, target, mat, o_del, e_del, o_ins, e_ins, xtra, size):
    """One ksw_u8 (size 1) / ksw_i16 (size 2) pass.  Returns [score, te, qe, score2, te2]."""
    P = 16 if size == 1 else 8
    qlen, tlen = len(query), len(target)
    L = (qlen + P - 1) // P
    ncol = L * P
    u8 = size == 1
    shift = _shift(mat)
    mx = max(max(mat), 0)
    minsc = xtra & 0xFFFF if xtra & KSW_XSUBO else 0x10000
    endsc = xtra & 0xFFFF if xtra & KSW_XSTOP else 0x10000
    oe_del, oe_ins = o_del + e_del, o_ins + e_ins
    H = [0] * ncol
    E = [0] * ncol
    gmax, te, qe = 0, -1, -1
    hmax_row = [0] * ncol
    b = []                       # [score, row]
    for i in range(tlen):
        t = target[i]
        Hn = [0] * ncol
        f = fx = hdiag = imax = 0
        for j in range(ncol):
            if j and j % L == 0:
                fx = max(fx, f)
                f = 0
            s = mat[t * 5 + query[j]] if j < qlen else 0
            if u8:
                m = max(min(hdiag + s + shift, 255) - shift, 0)
            else:
                m = max(min(hdiag + s, 32767), -32768)
            h1 = max(m, E[j], f)
            imax = max(imax, h1)
            Hn[j] = max(h1, fx)
            E[j] = max(E[j] - e_del, h1 - oe_del, 0)
            f = max(f - e_ins, h1 - oe_ins, 0)
            fx -= e_ins
            hdiag = H[j]
        H = Hn
        if imax >= minsc:
            if not b or b[-1][1] + 1 != i:
                b.append([imax, i])
            elif b[-1][0] < imax:
                b[-1] = [imax, i]
        if imax > gmax:
            gmax, te = imax, i
            hmax_row = list(Hn)
            if (u8 and gmax + shift >= 255) or gmax >= endsc:
                break
    score = 255 if (u8 and gmax + shift >= 255) else gmax
    score2 = te2 = -1
    if not (u8 and score == 255):
        if ncol:
            top = max(hmax_row)
            qe = min(j for j in range(ncol) if hmax_row[j] == top)
        if b:
            w = (score + mx - 1) // mx
            low, high = te - w, te + w
            for sc, row in b:
                if (row < low or row > high) and sc > score2:
                    score2, te2 = sc, row
    return [score, te, qe, score2, te2]


def ksw_align2(query, target, mat, o_del, e_del, o_ins, e_ins, xtra):
    """kswr_t (score, te, qe, score2, te2, tb, qb) of upstream ksw_align2 (qry == NULL)."""
    size = 1 if xtra & KSW_XBYTE else 2
    score, te, qe, score2, te2 = ksw_local(list(query), list(target), mat, o_del, e_del, o_ins, e_ins,
                                           xtra, size)
    tb = qb = -1
    if (xtra & KSW_XSTART) and not ((xtra & KSW_XSUBO) and score < (xtra & 0xFFFF)):
        rq = list(query[:qe + 1])[::-1]
        rt = list(target[:te + 1])[::-1] + list(target[te + 1:])
        rs, rte, rqe, _, _ = ksw_local(rq, rt, mat, o_del, e_del, o_ins, e_ins, KSW_XSTOP | score, size)
        if rs == score:
            tb, qb = te - rte, qe - rqe
    return [score, te, qe, score2, te2, tb, qb]
