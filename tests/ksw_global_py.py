"""Independent formulation of upstream ksw_global2 (banded global alignment + CIGAR) for the
oracle cross-check -- TEST INFRASTRUCTURE (tests/test_global.py).

Where oracle/ksw_global_ref.c restates upstream's single-row `eh[]` buffer literally, this
module writes the same recurrence as explicit band matrices over cells (i, j) with
max(i - w, 0) <= j < min(i + w + 1, qlen):

    M(i, j) = Hd(i - 1, j - 1) + S(i, j)    Hd: H on the diagonal, with the virtual row -1
                                            (0, then -(o_ins + e_ins j) up to w) and the column
                                            boundary H(i, -1) = -(o_del + e_del (i + 1))
    E(i, j) = E'(i - 1, j) if (i - 1, j) is a band cell, else -inf
    F(i, j) = F'(i, j - 1) if (i, j - 1) is a band cell, else -inf
    H = max(M, E, F), direction 0 / 1 / 2 with ties to M, then E
    E' = max(E - e_del, M - oe_del),  F' = max(F - e_ins, M - oe_ins), extension bits on '>'

and reads the score off the last row.  The traceback state machine (upstream's `which`) is
shared by construction: it is what defines the CIGAR.  Small sizes only (pure Python).
"""

NEG = -0x40000000


def band(i, w, qlen):
    return max(i - w, 0), min(i + w + 1, qlen)


def ksw_global2(q, t, mat, o_del, e_del, o_ins, e_ins, w):
    """-> (score, cigar as [(op, len)], ops M=0, I=1, D=2); raises for the undefined geometry."""
    Q, T = len(q), len(t)
    oe_del, oe_ins = o_del + e_del, o_ins + e_ins
    H, Ep, Fp, Z = {}, {}, {}, {}

    def hd(i, j):
        if i < 0:
            return 0 if j < 0 else (-(o_ins + e_ins * (j + 1)) if j + 1 <= w else NEG)
        if j < 0:
            return -(o_del + e_del * (i + 1))
        return H[i, j]

    def inb(i, j):
        lo, hi = band(i, w, Q)
        return i >= 0 and lo <= j < hi

    for i in range(T):
        lo, hi = band(i, w, Q)
        for j in range(lo, hi):
            m = hd(i - 1, j - 1) + mat[t[i] * 5 + q[j]]
            e = Ep[i - 1, j] if inb(i - 1, j) else NEG
            f = Fp[i, j - 1] if inb(i, j - 1) else NEG
            h, d = (m, 0) if m >= e else (e, 1)
            h, d = (h, d) if h >= f else (f, 2)
            H[i, j] = h
            Ep[i, j] = max(e - e_del, m - oe_del)
            Fp[i, j] = max(f - e_ins, m - oe_ins)
            Z[i, j] = d | (4 if e - e_del > m - oe_del else 0) | (8 if f - e_ins > m - oe_ins else 0)
    if T == 0:
        score = 0 if Q == 0 else (-(o_ins + e_ins * Q) if Q <= w else NEG)
    else:
        lo, hi = band(T - 1, w, Q)
        if hi < Q:
            score = 0 if Q == 0 else (-(o_ins + e_ins * Q) if Q <= w else NEG)
        elif lo < hi:
            score = H[T - 1, Q - 1]
        else:
            score = -(o_del + e_del * T) if lo == 0 else NEG

    ops = []

    def push(op, ln):
        if ops and ops[-1][0] == op:
            ops[-1][1] += ln
        else:
            ops.append([op, ln])

    i, k, which = T - 1, min(T + w, Q) - 1, 0
    if i >= 0 and k >= 0 and not inb(i, k):
        raise ValueError("traceback start outside the band (qlen < tlen - w)")
    while i >= 0 and k >= 0:
        z = Z[i, k]
        which = (z & 3) if which == 0 else ((z >> 2) & 1 if which == 1 else (2 if z & 8 else 0))
        if which == 0:
            push(0, 1); i -= 1; k -= 1
        elif which == 1:
            push(2, 1); i -= 1
        else:
            push(1, 1); k -= 1
    if i >= 0:
        push(2, i + 1)
    if k >= 0:
        push(1, k + 1)
    return score, [tuple(o) for o in reversed(ops)]


def rescore(q, t, mat, o_del, e_del, o_ins, e_ins, cigar):
    """Score of the alignment a CIGAR describes (affine gaps, one open per run)."""
    i = j = sc = 0
    for op, ln in cigar:
        if op == 0:
            for _ in range(ln):
                sc += mat[t[i] * 5 + q[j]]
                i += 1
                j += 1
        elif op == 1:
            sc -= o_ins + e_ins * ln
            j += ln
        else:
            sc -= o_del + e_del * ln
            i += ln
    return sc, i, j


def gen_cigar_w(l_query, rlen, w_, a, o_del, e_del, o_ins, e_ins):
    """bwa_gen_cigar2's band width (src/bwa.cpp) for a query of l_query vs a ref span of rlen."""
    max_ins = int(float(((l_query + 1) >> 1) * a - o_ins) / e_ins + 1.0)
    max_del = int(float(((l_query + 1) >> 1) * a - o_del) / e_del + 1.0)
    max_gap = max(max(max_ins, max_del), 1)
    w = (max_gap + abs(rlen - l_query) + 1) >> 1
    w = min(w, w_)
    return max(w, abs(rlen - l_query) + 3)
