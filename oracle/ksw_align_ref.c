/*
 * ksw_align_ref.c -- TEST INFRASTRUCTURE (the CPU oracle of the mate-rescue batch, SURVEY.md
 * §8(f) row 2).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 *
 * A literal restatement of upstream's local Smith-Waterman used for mate rescue:
 * ksw_qinit / ksw_u8 / ksw_i16 / ksw_align2 in src/ksw.cpp (bwa's ksw.c), the scalar function
 * the fork falls back to for every 8-bit mate-rescue pair (docs-archive/WEEK2_STATUS.md:80-90,
 * docs-archive/PROJECT_SUMMARY.md:90-99, docs-archive/AWS_VALIDATION_SUCCESS.md:100-117) and
 * whose kswr_t results the batched kswv::getScores8/16 replaces
 * (docs-archive/INTEGRATION_COMPLETE.md:49-112, docs-archive/ARM-BATCHED-SAM-PLAN.md:34).
 * No ksw.cpp / kswv.cpp ships in /root/reference: the algorithm is restated from upstream
 * (bwa 0.7.17 ksw.c, bwa-mem2 v2.2.1 ksw.cpp) [UPSTREAM-RECALL, SURVEY.md row 3]; parity is
 * unpinned by reference fixtures (none exist for this path) and is pinned instead by an
 * independent non-striped Python formulation (tests/ksw_align_py.py).
 *
 * The SSE2 kernels are STRIPED (Farrar): query position k lives in vector k % slen, lane
 * k / slen, with slen = ceil(qlen / P), P = 16 (u8) or 8 (i16).  The result depends on the
 * striping in one place -- E(i+1, j) is computed from H before the lazy-F loop propagates F
 * across segment boundaries ("we disallow adjacent insertion and then deletion") -- so this
 * oracle keeps the striped layout: a vector is an array of P lanes, and every SSE operation
 * is restated lane by lane (adds/subs saturating exactly as _mm_adds_epu8 / _mm_subs_epu8 /
 * _mm_adds_epi16 / _mm_subs_epu16).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define KSW_XBYTE  0x10000
#define KSW_XSTOP  0x20000
#define KSW_XSUBO  0x40000
#define KSW_XSTART 0x80000

typedef struct { int32_t score, te, qe, score2, te2, tb, qb; } okswr_t;

typedef struct {               /* kswq_t */
    int qlen, slen, size, P;   /* size 1: u8 (P 16), size 2: i16 (P 8)  */
    int shift, mdiff, max;
    int *qp;                   /* [m][slen][P] profile                   */
} oqprof_t;

static inline int clampi(int x, int lo, int hi) { return x < lo ? lo : (x > hi ? hi : x); }
static inline int maxi(int a, int b) { return a > b ? a : b; }

/* ksw_qinit: shift = -min(mat) as uint8 (u8 only), mdiff = max(mat) + shift, max = max(mat, 0);
 * profile entry (lane l, vector i) = mat[a][query[i + l*slen]] (0 past qlen) [+ shift for u8]. */
static void oqinit(oqprof_t *q, int size, int qlen, const uint8_t *query, int m, const int8_t *mat)
{
    q->size = size;
    q->P = size == 1 ? 16 : 8;
    q->qlen = qlen;
    q->slen = (qlen + q->P - 1) / q->P;
    int mn = 127, mx = 0;
    for (int a = 0; a < m * m; ++a) {
        if (mat[a] < mn) mn = mat[a];
        if (mat[a] > mx) mx = mat[a];
    }
    q->max = mx;
    q->shift = (uint8_t)(256 - (uint8_t)(int8_t)mn);
    q->mdiff = mx + q->shift;
    const int P = q->P, slen = q->slen;
    q->qp = (int *)malloc(sizeof(int) * (size_t)m * (slen ? slen : 1) * P);
    int *t = q->qp;
    for (int a = 0; a < m; ++a) {
        const int8_t *ma = mat + a * m;
        for (int i = 0; i < slen; ++i)
            for (int l = 0; l < P; ++l) {
                const int k = i + l * slen;
                int v = k >= qlen ? 0 : ma[query[k]];
                *t++ = size == 1 ? (uint8_t)(v + q->shift) : v;
            }
    }
}

typedef struct { uint64_t *a; int n, m; } obarr_t;

static void bpush(obarr_t *b, int imax, int i)
{
    /* ksw_u8/ksw_i16 "write the b array": extend the last entry only when its row is i-1 */
    if (b->n == 0 || (int32_t)b->a[b->n - 1] + 1 != i) {
        if (b->n == b->m) {
            b->m = b->m ? b->m << 1 : 8;
            b->a = (uint64_t *)realloc(b->a, 8 * (size_t)b->m);
        }
        b->a[b->n++] = (uint64_t)imax << 32 | (uint32_t)i;
    } else if ((int)(b->a[b->n - 1] >> 32) < imax) {
        b->a[b->n - 1] = (uint64_t)imax << 32 | (uint32_t)i;
    }
}

/* ksw_u8 (size 1) and ksw_i16 (size 2) in one body; the differences are the lane count, the
 * saturation of H (u8: biased by shift, capped at 255; i16: signed 16-bit) and the u8 stop at
 * gmax + shift >= 255. */
static okswr_t oksw_striped(const oqprof_t *q, int tlen, const uint8_t *target, int o_del, int e_del,
                            int o_ins, int e_ins, int xtra)
{
    const int P = q->P, slen = q->slen, u8 = q->size == 1;
    const int minsc = (xtra & KSW_XSUBO) ? xtra & 0xffff : 0x10000;
    const int endsc = (xtra & KSW_XSTOP) ? xtra & 0xffff : 0x10000;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    const int hi = u8 ? 255 : 32767, lo = u8 ? 0 : -32768;
    okswr_t r = {0, -1, -1, -1, -1, -1, -1};
    const int nv = slen ? slen : 1;
    int *H0 = (int *)calloc((size_t)nv * P, sizeof(int)), *H1 = (int *)calloc((size_t)nv * P, sizeof(int));
    int *E = (int *)calloc((size_t)nv * P, sizeof(int)), *Hmax = (int *)calloc((size_t)nv * P, sizeof(int));
    int f[16], mxv[16], h[16], t[16], e[16];
    obarr_t b = {0, 0, 0};
    int gmax = 0, te = -1;
#define SUBS(x, y) maxi((x) - (y), 0)                 /* _mm_subs_epu8 / _mm_subs_epu16 */
    for (int i = 0; i < tlen; ++i) {
        const int *S = q->qp + (size_t)target[i] * slen * P;
        for (int l = 0; l < P; ++l) f[l] = mxv[l] = 0;
        /* h = H0[slen-1] shifted up one lane: H(i-1, -1) = 0 enters lane 0 */
        h[0] = 0;
        for (int l = 1; l < P; ++l) h[l] = slen ? H0[(slen - 1) * P + l - 1] : 0;
        for (int j = 0; j < slen; ++j) {
            for (int l = 0; l < P; ++l) {
                int v;
                if (u8) v = SUBS(clampi(h[l] + S[j * P + l], 0, 255), q->shift);   /* adds_epu8; subs_epu8 */
                else    v = clampi(h[l] + S[j * P + l], lo, hi);                    /* adds_epi16 */
                e[l] = E[j * P + l];
                v = maxi(v, e[l]);
                v = maxi(v, f[l]);
                mxv[l] = maxi(mxv[l], v);
                H1[j * P + l] = v;
                h[l] = v;
            }
            for (int l = 0; l < P; ++l) {
                e[l] = SUBS(e[l], e_del);
                t[l] = SUBS(h[l], oe_del);
                E[j * P + l] = maxi(e[l], t[l]);
                f[l] = SUBS(f[l], e_ins);
                t[l] = SUBS(h[l], oe_ins);
                f[l] = maxi(f[l], t[l]);
                h[l] = H0[j * P + l];
            }
        }
        /* lazy-F loop (SWPS3): at most P shifts of the F vector across segment boundaries */
        for (int k = 0; k < P && slen; ++k) {
            for (int l = P - 1; l > 0; --l) f[l] = f[l - 1];
            f[0] = 0;
            for (int j = 0; j < slen; ++j) {
                int done = 1;
                for (int l = 0; l < P; ++l) {
                    int v = maxi(H1[j * P + l], f[l]);
                    H1[j * P + l] = v;
                    v = SUBS(v, oe_ins);
                    f[l] = SUBS(f[l], e_ins);
                    if (SUBS(f[l], v) != 0) done = 0;      /* u8: cmpeq(subs(f,h),0); i16: !(f > h) */
                }
                if (done) goto end_loop;
            }
        }
    end_loop:;
        int imax = 0;
        for (int l = 0; l < P; ++l) imax = maxi(imax, mxv[l]);
        if (imax >= minsc) bpush(&b, imax, i);
        if (imax > gmax) {
            gmax = imax;
            te = i;
            memcpy(Hmax, H1, sizeof(int) * (size_t)nv * P);
            if ((u8 && gmax + q->shift >= 255) || gmax >= endsc) break;
        }
        int *tmp = H0; H0 = H1; H1 = tmp;
    }
#undef SUBS
    r.score = (u8 && gmax + q->shift >= 255) ? 255 : gmax;
    r.te = te;
    if (r.score != 255 || !u8) {
        int mx = -1, qlen = slen * P;
        for (int i = 0; i < qlen; ++i) {       /* memory order: vector i / P, lane i % P */
            const int v = Hmax[i], pos = i / P + (i % P) * slen;
            if (v > mx) mx = v, r.qe = pos;
            else if (v == mx && pos < r.qe) r.qe = pos;
        }
        if (b.n) {
            const int w = (r.score + q->max - 1) / q->max;
            const int low = te - w, high = te + w;
            for (int i = 0; i < b.n; ++i) {
                const int e2 = (int32_t)b.a[i];
                if ((e2 < low || e2 > high) && (int)(b.a[i] >> 32) > r.score2)
                    r.score2 = (int)(b.a[i] >> 32), r.te2 = e2;
            }
        }
    }
    free(b.a); free(H0); free(H1); free(E); free(Hmax);
    return r;
}

static void revseq(int l, uint8_t *s)
{
    for (int i = 0; i < l >> 1; ++i) {
        const uint8_t t = s[i];
        s[i] = s[l - 1 - i];
        s[l - 1 - i] = t;
    }
}

/* ksw_align2 (qry == NULL): forward pass; with KSW_XSTART (and, under KSW_XSUBO, score >=
 * minsc) a second pass over the reversed prefixes query[0, qe] / target[0, te] stopping at
 * the forward score gives tb / qb when it reproduces that score.  The reverse pass is run
 * on tlen rows of the partially reversed target, as upstream does. */
okswr_t oracle_ksw_align2(int qlen, const uint8_t *query0, int tlen, const uint8_t *target0, int m,
                          const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int xtra)
{
    uint8_t *query = (uint8_t *)malloc(qlen > 0 ? qlen : 1), *target = (uint8_t *)malloc(tlen > 0 ? tlen : 1);
    if (qlen > 0) memcpy(query, query0, qlen);
    if (tlen > 0) memcpy(target, target0, tlen);
    oqprof_t q;
    const int size = (xtra & KSW_XBYTE) ? 1 : 2;
    oqinit(&q, size, qlen, query, m, mat);
    okswr_t r = oksw_striped(&q, tlen, target, o_del, e_del, o_ins, e_ins, xtra);
    free(q.qp);
    if ((xtra & KSW_XSTART) && !((xtra & KSW_XSUBO) && r.score < (xtra & 0xffff))) {
        revseq(r.qe + 1, query);
        revseq(r.te + 1, target);
        oqinit(&q, size, r.qe + 1, query, m, mat);
        okswr_t rr = oksw_striped(&q, tlen, target, o_del, e_del, o_ins, e_ins, KSW_XSTOP | r.score);
        free(q.qp);
        if (r.score == rr.score) r.tb = r.te - rr.te, r.qb = r.qe - rr.qe;
    }
    free(query);
    free(target);
    return r;
}

/* Batch form over SeqPairs (idr, idq, len1 = target, len2 = query, h0 = xtra), results in
 * aln[i]; the layout the batched kswv::getScores8/16 takes.  nthreads host threads. */
typedef struct {
    int32_t idr, idq, id, len1, len2, h0, seqid, regid, score, tle, gtle, qle, gscore, max_off;
} oseqpair_t;

typedef struct {
    const oseqpair_t *p; const uint8_t *ref, *qer; okswr_t *aln; int n, nth, t;
    const int8_t *mat; int o_del, e_del, o_ins, e_ins;
} ojob_t;

static void *oworker(void *arg)
{
    ojob_t *j = (ojob_t *)arg;
    for (int i = j->t; i < j->n; i += j->nth) {
        const oseqpair_t *s = &j->p[i];
        j->aln[i] = oracle_ksw_align2(s->len2, j->qer + s->idq, s->len1, j->ref + s->idr, 5, j->mat, j->o_del,
                                      j->e_del, j->o_ins, j->e_ins, s->h0);
    }
    return 0;
}

void oracle_ksw_align2_batch(const void *pairs, const uint8_t *ref, const uint8_t *qer, int n,
                             const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, void *aln,
                             int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 512) nthreads = 512;
    pthread_t th[512];
    ojob_t jb[512];
    for (int t = 0; t < nthreads; ++t) {
        jb[t] = (ojob_t){(const oseqpair_t *)pairs, ref, qer, (okswr_t *)aln, n, nthreads, t, mat, o_del,
                         e_del, o_ins, e_ins};
        pthread_create(&th[t], 0, oworker, &jb[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], 0);
}
