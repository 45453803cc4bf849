"""Seeded SeqPair batch generators for the parity tests (numpy; no GPU, no oracle).

Every generator returns (pairs, ref, qer): `pairs` a structured array in the upstream
SeqPair layout (oracle.SEQPAIR_DTYPE mirror below), `ref` / `qer` the concatenated
1-byte-per-base code buffers (0..3 = ACGT, 4 = N) that idr / idq index into -- i.e. the
exact arguments of getScores16(pairs, seqBufRef, seqBufQer, n, nthreads, w).
"""

from __future__ import annotations

import numpy as np

SEQPAIR_DTYPE = np.dtype(
    [(n, "<i4") for n in ("idr", "idq", "id", "len1", "len2", "h0", "seqid", "regid",
                          "score", "tle", "gtle", "qle", "gscore", "max_off")]
)
OUT_FIELDS = ("score", "tle", "gtle", "qle", "gscore", "max_off")


def mutate(rng, src, qlen, p_sub, p_indel, p_n=0.0):
    """Query derived from `src`: substitutions, 1-3 bp indels, optional N."""
    out = []
    i = 0
    while len(out) < qlen:
        u = rng.random()
        if u < p_indel:
            ln = int(rng.integers(1, 4))
            if rng.random() < 0.5:
                out.extend(int(x) for x in rng.integers(0, 4, ln))
            else:
                i += ln
            continue
        b = int(src[i]) if i < len(src) else int(rng.integers(0, 4))
        i += 1
        if u < p_indel + p_sub and b < 4:
            b = (b + int(rng.integers(1, 4))) & 3
        if p_n and rng.random() < p_n:
            b = 4
        out.append(b)
    return np.array(out[:qlen], dtype=np.uint8)


def assemble(items, seqid_base=0):
    """items: list of (ref_codes, query_codes, h0)."""
    n = len(items)
    pairs = np.zeros(n, dtype=SEQPAIR_DTYPE)
    rl = [len(r) for r, _, _ in items]
    ql = [len(q) for _, q, _ in items]
    ref = np.zeros(max(1, sum(rl)), dtype=np.uint8)
    qer = np.zeros(max(1, sum(ql)), dtype=np.uint8)
    ro = qo = 0
    for k, (r, q, h0) in enumerate(items):
        ref[ro:ro + len(r)] = r
        qer[qo:qo + len(q)] = q
        p = pairs[k]
        p["idr"], p["idq"], p["id"] = ro, qo, k
        p["len1"], p["len2"], p["h0"] = len(r), len(q), h0
        p["seqid"], p["regid"] = seqid_base + k, 0
        ro += len(r)
        qo += len(q)
    return pairs, ref, qer


def random_pairs(n, seed, tlen=(0, 320), qlen=(0, 170), h0=(1, 150), p_sub=(0.0, 0.15),
                 p_indel=(0.0, 0.05), p_unrelated=0.1, p_n=0.02, related_prefix=True):
    """Mixed-shape batch: lengths uniform in the given inclusive ranges."""
    rng = np.random.default_rng(seed)
    items = []
    for _ in range(n):
        T = int(rng.integers(tlen[0], tlen[1] + 1))
        Q = int(rng.integers(qlen[0], qlen[1] + 1))
        r = rng.integers(0, 4, T).astype(np.uint8)
        if p_n:
            r[rng.random(T) < p_n] = 4
        if rng.random() < p_unrelated or not related_prefix:
            q = rng.integers(0, 4, Q).astype(np.uint8)
        else:
            q = mutate(rng, r, Q, rng.uniform(*p_sub), rng.uniform(*p_indel), p_n * 0.5)
        items.append((r, q, int(rng.integers(h0[0], h0[1] + 1))))
    return assemble(items)


def c2_like(n, seed, tlen=300, qlen=150, h0=(19, 100)):
    """Same distribution as the bench workload (bsw_synth.c), generated in numpy."""
    rng = np.random.default_rng(seed)
    items = []
    for _ in range(n):
        r = rng.integers(0, 4, tlen).astype(np.uint8)
        r[rng.random(tlen) < 0.001] = 4
        if rng.random() < 0.1:
            q = rng.integers(0, 4, qlen).astype(np.uint8)
        else:
            q = mutate(rng, r, qlen, 0.02, 0.002)
        items.append((r, q, int(rng.integers(h0[0], h0[1] + 1))))
    return assemble(items)


def edge_pairs(seed=7):
    """Edge cases the reference's bug history and SURVEY.md §8(c) call out: empty and
    length-1 sequences, lengths around 16/32/64/128 lane and MAX_SEQ_LEN8 boundaries,
    all-N, repeats, exact matches, h0 extremes."""
    rng = np.random.default_rng(seed)
    items = []
    lens = [0, 1, 2, 3, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 150, 159, 160]
    for L in lens:
        r = rng.integers(0, 4, L).astype(np.uint8)
        items.append((r, r.copy(), 20))                          # identical
        items.append((r, rng.integers(0, 4, L).astype(np.uint8), 4))  # unrelated, low h0
        items.append((np.concatenate([r, rng.integers(0, 4, 30).astype(np.uint8)]), r.copy(), 30))
        items.append((r, np.full(L, 4, np.uint8), 50))           # all-N query
        items.append((np.full(L, 4, np.uint8), r.copy(), 50))    # all-N ref
    for L in (40, 100, 150):
        rep = np.tile(np.array([0, 1], np.uint8), L)[:L]
        items.append((rep, rep[1:].copy(), 60))                  # repeats / ties
        items.append((rep, rep.copy(), 1))
        rr = rng.integers(0, 4, 2 * L).astype(np.uint8)
        items.append((rr, mutate(rng, rr, L, 0.05, 0.02), 250))  # large h0
        items.append((rr, mutate(rng, rr, L, 0.05, 0.02), 1))    # tiny h0
    return assemble(items)


def pairs_from_shapes(shapes, seed, p_unrelated=0.2):
    """shapes: list of (tlen, qlen, h0); related (mutated-prefix) queries unless unrelated."""
    rng = np.random.default_rng(seed)
    items = []
    for T, Q, h0 in shapes:
        r = rng.integers(0, 4, T).astype(np.uint8)
        if rng.random() < p_unrelated:
            q = rng.integers(0, 4, Q).astype(np.uint8)
        else:
            q = mutate(rng, r, Q, rng.uniform(0.0, 0.08), rng.uniform(0.0, 0.03), 0.01)
        items.append((r, q, int(h0)))
    return assemble(items)


def repeat_pairs(n, seed, L=(20, 160), h0=(1, 120)):
    """Tandem repeats (period 1..6 motifs, microsatellites) with light mutation: equal-score
    paths everywhere, so the last-index tie rules (row max mj, gscore's max_ie) decide."""
    rng = np.random.default_rng(seed)
    items = []
    for _ in range(n):
        per = int(rng.integers(1, 7))
        motif = rng.integers(0, 4, per).astype(np.uint8)
        Q = int(rng.integers(L[0], L[1] + 1))
        T = Q + int(rng.integers(0, 60))
        r = np.tile(motif, T // per + 2)[int(rng.integers(0, per)):][:T].copy()
        q = np.tile(motif, Q // per + 2)[:Q].copy()
        if rng.random() < 0.5:
            q = mutate(rng, q, Q, 0.03, 0.01)
        items.append((r, q, int(rng.integers(h0[0], h0[1] + 1))))
    return assemble(items)
