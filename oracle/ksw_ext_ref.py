"""CPU ORACLE, Python transcription (test infrastructure only; never shipped to the product).

An independent restatement of `ksw_extend2` (upstream bwa-mem2 v2.2.1 `src/ksw.cpp`,
= lh3/bwa ksw.c) written directly from SURVEY.md Appendix A, rules A.1-A.6, so that a
transcription slip in oracle/ksw_ext_ref.c shows up as a disagreement between the two.
Pure-Python loops: use it only on small cases (tests/test_oracle.py).

PARITY UNPINNED by the reference: /root/reference holds no source, fixtures or tests for
this path; see oracle/ksw_ext_ref.c's header for how the oracle is pinned.
"""

from __future__ import annotations

import math


def bwa_fill_scmat(a: int = 1, b: int = 4, ambig: int = -1) -> list[int]:
    """bwa's bwa_fill_scmat: a on the ACGT diagonal, -b off it, `ambig` on row/col N."""
    mat = []
    for t in range(5):
        for q in range(5):
            if t == 4 or q == 4:
                mat.append(ambig)
            else:
                mat.append(a if t == q else -b)
    return mat


def ksw_extend2(query, target, mat, o_del, e_del, o_ins, e_ins, w, end_bonus, zdrop, h0):
    """Returns (score, qle, tle, gtle, gscore, max_off) -- SURVEY.md A.6 order remapped to
    the SeqPair output names."""
    qlen, tlen = len(query), len(target)
    # A.1 row buffer, qlen+2 entries (upstream writes eh[1] even when qlen == 0)
    H = [0] * (qlen + 2)
    E = [0] * (qlen + 2)
    H[0] = h0
    H[1] = max(h0 - (o_ins + e_ins), 0)
    j = 2
    while j <= qlen and H[j - 1] > e_ins:
        H[j] = H[j - 1] - e_ins
        j += 1
    # A.2 band cap (C semantics: double division, truncation toward zero)
    maxsc = max(0, max(mat))
    max_ins = max(int(math.trunc((qlen * maxsc + end_bonus - o_ins) / e_ins + 1.0)), 1)
    w = min(w, max_ins)
    max_del = max(int(math.trunc((qlen * maxsc + end_bonus - o_del) / e_del + 1.0)), 1)
    w = min(w, max_del)
    # A.3 state
    best, best_i, best_j = h0, -1, -1
    max_ie, gscore, max_off = -1, -1, 0
    beg, end = 0, qlen
    for i in range(tlen):
        row = mat[target[i] * 5: target[i] * 5 + 5]
        beg = max(beg, i - w)
        end = min(end, i + w + 1, qlen)
        h1 = max(h0 - (o_del + e_del * (i + 1)), 0) if beg == 0 else 0
        f = 0
        m = 0
        mj = -1
        for j in range(beg, end):
            M, e = H[j], E[j]
            H[j] = h1
            M = M + row[query[j]] if M != 0 else 0
            h = max(M, e, f)
            h1 = h
            if not (m > h):
                mj = j
            m = max(m, h)
            e = max(e - e_del, M - (o_del + e_del), 0)
            E[j] = e
            f = max(f - e_ins, M - (o_ins + e_ins), 0)
        H[end] = h1
        E[end] = 0
        jx = end if beg < end else beg
        if jx == qlen:
            if not (gscore > h1):
                max_ie = i
            gscore = max(gscore, h1)
        if m == 0:
            break
        if m > best:
            best, best_i, best_j = m, i, mj
            max_off = max(max_off, abs(mj - i))
        elif zdrop > 0:
            di, dj = i - best_i, mj - best_j
            if di > dj:
                if best - m - (di - dj) * e_del > zdrop:
                    break
            elif best - m - (dj - di) * e_ins > zdrop:
                break
        j = beg
        while j < end and H[j] == 0 and E[j] == 0:
            j += 1
        beg = j
        j = end
        while j >= beg and H[j] == 0 and E[j] == 0:
            j -= 1
        end = min(j + 2, qlen)
    return best, best_j + 1, best_i + 1, max_ie + 1, gscore, max_off
