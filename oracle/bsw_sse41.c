/*
 * oracle/bsw_sse41.c -- CPU BASELINE (test / bench infrastructure only).
 *
 * A restatement of the reference's CPU path for this hot loop: upstream bwa-mem2
 * `BandedPairWiseSW::getScores16` -> `smithWatermanBatchWrapper16` ->
 * `smithWaterman128_16` (SSE2/SSE4.1 section of src/bandedSWA.cpp, lines 3361-4872 per
 * docs-archive/ARM-BATCHED-SAM-PLAN.md:60-64), whose design the reference documents:
 *   - sort pairs by length, pad to a multiple of the SIMD width with len=0 pairs
 *     (docs-archive/WEEK1_WRAPPER_COMPLETE.md:55-58, docs-archive/WEEK2_STATUS.md:44-60);
 *   - one pair per SIMD lane, 8 x int16 lanes for the 16-bit path
 *     (docs-archive/ARM-BATCHED-SAM-PLAN.md:129-134);
 *   - AoS -> SoA transpose of both sequences with DUMMY padding
 *     (docs-archive/WEEK1_WRAPPER_COMPLETE.md:64-83);
 *   - boundary rows from h0 and per-lane band min(w, max_ins, max_del)
 *     (docs-archive/WEEK1_WRAPPER_COMPLETE.md:85-118);
 *   - threads over batches (`omp for schedule(dynamic, 128)` upstream; pthreads here).
 * The upstream C++ is not available, so this is NOT the upstream binary:
 * it is the same design, written here, and it must reproduce the scalar oracle
 * (oracle/ksw_ext_ref.c) bit for bit -- tests/test_oracle.py checks that.  Per-lane
 * semantics follow SURVEY.md Appendix A with two exact simplifications proved in
 * the left band edge is max(0, i-w) (A.9 (ii)) and the right edge after a
 * row is min(lastH + 3, qlen), lastH = last column with H(i,j) > 0.
 *
 * bench.py reports it as cpu_baseline kind "port".
 */
#include <smmintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../include/bsw_seqpair.h"

#define W16 8
#define DUMMY1 99
#define DUMMY2 100

typedef struct {
    int32_t o_del, e_del, o_ins, e_ins, zdrop, end_bonus;
    int8_t mat[25];
} sse_params_t;

int oracle_ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target,
                       int m, const int8_t *mat, int o_del, int e_del, int o_ins,
                       int e_ins, int w, int end_bonus, int zdrop, int h0, int *_qle,
                       int *_tle, int *_gtle, int *_gscore, int *_max_off);

static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int imin(int a, int b) { return a < b ? a : b; }

/* per-lane band cap (A.2), integer form of (int)((double)N / e + 1.) */
static int band_cap(const sse_params_t *p, int qlen, int w, int maxsc)
{
    int n_ins = qlen * maxsc + p->end_bonus - p->o_ins;
    int n_del = qlen * maxsc + p->end_bonus - p->o_del;
    int mi = (n_ins + p->e_ins) / p->e_ins, md = (n_del + p->e_del) / p->e_del;
    mi = mi > 1 ? mi : 1;
    md = md > 1 ? md : 1;
    w = w < mi ? w : mi;
    return w < md ? w : md;
}

typedef struct {
    int16_t *s1, *s2;  /* SoA sequences [len][W16] */
    int16_t *H, *E;    /* eh row [qlen+1][W16]     */
    int cap;           /* allocated rows           */
} sse_scratch_t;

static void scratch_reserve(sse_scratch_t *s, int rows)
{
    if (rows <= s->cap) return;
    free(s->s1); free(s->s2); free(s->H); free(s->E);
    s->cap = rows;
    size_t b = (size_t)rows * W16 * sizeof(int16_t);
    s->s1 = (int16_t *)aligned_alloc(16, b);
    s->s2 = (int16_t *)aligned_alloc(16, b);
    s->H = (int16_t *)aligned_alloc(16, b);
    s->E = (int16_t *)aligned_alloc(16, b);
}

/* Align one batch of up to 8 pairs (one per lane). */
static void batch16(const sse_params_t *p, SeqPair **bp, int nb, const uint8_t *ref,
                    const uint8_t *qer, int w, int maxsc, sse_scratch_t *sc)
{
    int maxT = 0, maxQ = 0;
    for (int l = 0; l < nb; ++l) { maxT = imax(maxT, bp[l]->len1); maxQ = imax(maxQ, bp[l]->len2); }
    scratch_reserve(sc, imax(maxT, maxQ) + 2);
    int16_t *S1 = sc->s1, *S2 = sc->s2, *H = sc->H, *E = sc->E;
    /* AoS -> SoA transpose with DUMMY padding; boundary row A.1 */
    int16_t wl[W16], qlen[W16], tlen[W16], h0v[W16];
    for (int l = 0; l < W16; ++l) {
        SeqPair *sp = l < nb ? bp[l] : NULL;
        int T = sp ? sp->len1 : 0, Q = sp ? sp->len2 : 0;
        const uint8_t *r = sp ? ref + sp->idr : NULL, *q = sp ? qer + sp->idq : NULL;
        for (int i = 0; i < maxT; ++i) S1[i * W16 + l] = i < T ? r[i] : DUMMY1;
        for (int j = 0; j < maxQ; ++j) S2[j * W16 + l] = j < Q ? q[j] : DUMMY2;
        int h0 = sp ? sp->h0 : 0;
        int oe_ins = p->o_ins + p->e_ins;
        for (int j = 0; j <= maxQ + 1; ++j) { H[j * W16 + l] = 0; E[j * W16 + l] = 0; }
        H[l] = (int16_t)h0;
        H[W16 + l] = (int16_t)(h0 > oe_ins ? h0 - oe_ins : 0);
        for (int j = 2; j <= Q && H[(j - 1) * W16 + l] > p->e_ins; ++j)
            H[j * W16 + l] = (int16_t)(H[(j - 1) * W16 + l] - p->e_ins);
        wl[l] = (int16_t)band_cap(p, Q, w, maxsc);
        qlen[l] = (int16_t)Q;
        tlen[l] = (int16_t)T;
        h0v[l] = (int16_t)h0;
    }
    /* per-lane scalar state */
    int best[W16], best_i[W16], best_j[W16], max_ie[W16], gsc[W16], moff[W16], endl[W16];
    int alive[W16];
    for (int l = 0; l < W16; ++l) {
        best[l] = h0v[l]; best_i[l] = best_j[l] = -1; max_ie[l] = -1; gsc[l] = -1; moff[l] = 0;
        endl[l] = qlen[l];
        alive[l] = l < nb && tlen[l] > 0;
    }
    const __m128i vzero = _mm_setzero_si128();
    const __m128i vmatch = _mm_set1_epi16(p->mat[0]);        /* a  (mat[A][A])  */
    const __m128i vmis = _mm_set1_epi16(p->mat[1]);          /* -b (mat[A][C])  */
    const __m128i vambig = _mm_set1_epi16(p->mat[4]);        /* N score         */
    const __m128i vfour = _mm_set1_epi16(4);
    const __m128i ve_del = _mm_set1_epi16((int16_t)p->e_del), ve_ins = _mm_set1_epi16((int16_t)p->e_ins);
    const __m128i voe_del = _mm_set1_epi16((int16_t)(p->o_del + p->e_del));
    const __m128i voe_ins = _mm_set1_epi16((int16_t)(p->o_ins + p->e_ins));
    const __m128i vone = _mm_set1_epi16(1);

    for (int i = 0; i < maxT; ++i) {
        int any = 0;
        int16_t begv[W16], endv[W16], h1v[W16], actv[W16];
        int ubeg = 1 << 30, uend = -1;
        for (int l = 0; l < W16; ++l) {
            int act = alive[l] && i < tlen[l];
            alive[l] = act;
            actv[l] = (int16_t)(act ? -1 : 0);
            int b = imax(0, i - wl[l]);
            int e = imin(imin(endl[l], i + wl[l] + 1), qlen[l]);
            endl[l] = e;
            begv[l] = (int16_t)b;
            endv[l] = (int16_t)(act ? e : -1);
            int h1 = 0;
            if (b == 0) { h1 = h0v[l] - (p->o_del + p->e_del * (i + 1)); h1 = h1 < 0 ? 0 : h1; }
            h1v[l] = (int16_t)h1;
            if (act) { any = 1; ubeg = imin(ubeg, b); uend = imax(uend, e); }
        }
        if (!any) break;
        __m128i vbeg = _mm_loadu_si128((const __m128i *)begv);
        __m128i vend = _mm_loadu_si128((const __m128i *)endv);
        __m128i vact = _mm_loadu_si128((const __m128i *)actv);
        __m128i h1 = _mm_loadu_si128((const __m128i *)h1v);
        __m128i f = vzero, m = vzero, mj = _mm_set1_epi16(-1), lastH = _mm_set1_epi16(-1);
        __m128i s1 = _mm_load_si128((const __m128i *)(S1 + i * W16));
        __m128i s1amb = _mm_cmpeq_epi16(s1, vfour);
        for (int j = ubeg; j <= uend; ++j) {
            __m128i vj = _mm_set1_epi16((int16_t)j);
            /* in-band: beg <= j < end ; at-end: j == end */
            __m128i in = _mm_and_si128(_mm_and_si128(vact, _mm_cmplt_epi16(vj, vend)),
                                       _mm_cmpgt_epi16(_mm_add_epi16(vj, vone), vbeg));
            __m128i atend = _mm_cmpeq_epi16(vj, vend);
            __m128i Hj = _mm_load_si128((const __m128i *)(H + j * W16));
            __m128i Ej = _mm_load_si128((const __m128i *)(E + j * W16));
            __m128i s2 = _mm_load_si128((const __m128i *)(S2 + j * W16));
            __m128i sbt = _mm_blendv_epi8(vmis, vmatch, _mm_cmpeq_epi16(s1, s2));
            sbt = _mm_blendv_epi8(sbt, vambig, _mm_or_si128(s1amb, _mm_cmpeq_epi16(s2, vfour)));
            __m128i M = _mm_andnot_si128(_mm_cmpeq_epi16(Hj, vzero), _mm_add_epi16(Hj, sbt));
            __m128i h = _mm_max_epi16(_mm_max_epi16(M, Ej), f);
            __m128i ge = _mm_and_si128(in, _mm_cmpgt_epi16(_mm_add_epi16(h, vone), m)); /* h >= m */
            mj = _mm_blendv_epi8(mj, vj, ge);
            m = _mm_blendv_epi8(m, h, ge);
            lastH = _mm_blendv_epi8(lastH, vj, _mm_and_si128(in, _mm_cmpgt_epi16(h, vzero)));
            __m128i t = _mm_max_epi16(_mm_sub_epi16(M, voe_del), vzero);
            __m128i e2 = _mm_max_epi16(_mm_sub_epi16(Ej, ve_del), t);
            t = _mm_max_epi16(_mm_sub_epi16(M, voe_ins), vzero);
            __m128i f2 = _mm_max_epi16(_mm_sub_epi16(f, ve_ins), t);
            /* eh[j].h = h1 (in band or at end); eh[j].e = e' in band, 0 at end */
            __m128i wr = _mm_or_si128(in, atend);
            _mm_store_si128((__m128i *)(H + j * W16), _mm_blendv_epi8(Hj, h1, wr));
            _mm_store_si128((__m128i *)(E + j * W16),
                            _mm_blendv_epi8(_mm_andnot_si128(atend, Ej), e2, in));
            h1 = _mm_blendv_epi8(h1, h, in);
            f = _mm_blendv_epi8(f, f2, in);
        }
        int16_t mv[W16], mjv[W16], lh[W16], h1o[W16];
        _mm_storeu_si128((__m128i *)mv, m);
        _mm_storeu_si128((__m128i *)mjv, mj);
        _mm_storeu_si128((__m128i *)lh, lastH);
        _mm_storeu_si128((__m128i *)h1o, h1);
        for (int l = 0; l < W16; ++l) {
            if (!alive[l]) continue;
            int hh = h1o[l], mm = mv[l], mjj = mjv[l];
            if (endl[l] == qlen[l]) {        /* jx == qlen (beg <= end always) */
                if (!(gsc[l] > hh)) max_ie[l] = i;
                gsc[l] = gsc[l] > hh ? gsc[l] : hh;
            }
            if (mm == 0) { alive[l] = 0; continue; }
            if (mm > best[l]) {
                best[l] = mm; best_i[l] = i; best_j[l] = mjj;
                int d = mjj - i; d = d < 0 ? -d : d;
                moff[l] = moff[l] > d ? moff[l] : d;
            } else if (p->zdrop > 0) {
                int di = i - best_i[l], dj = mjj - best_j[l];
                if (di > dj) {
                    if (best[l] - mm - (di - dj) * p->e_del > p->zdrop) { alive[l] = 0; continue; }
                } else if (best[l] - mm - (dj - di) * p->e_ins > p->zdrop) { alive[l] = 0; continue; }
            }
            endl[l] = imin(lh[l] + 3, qlen[l]);
        }
    }
    for (int l = 0; l < nb; ++l) {
        SeqPair *sp = bp[l];
        sp->score = best[l];
        sp->qle = best_j[l] + 1;
        sp->tle = best_i[l] + 1;
        sp->gtle = max_ie[l] + 1;
        sp->gscore = gsc[l];
        sp->max_off = moff[l];
    }
}

typedef struct {
    const sse_params_t *p;
    SeqPair **order;
    int32_t n, w, maxsc;
    const uint8_t *ref, *qer;
    volatile int32_t *next;
} sse_job_t;

static void *sse_worker(void *arg)
{
    sse_job_t *jb = (sse_job_t *)arg;
    sse_scratch_t sc = {0};
    const int chunk = 16 * W16;   /* pairs per work item (upstream: dynamic, 128) */
    for (;;) {
        int32_t a = __sync_fetch_and_add(jb->next, chunk);
        if (a >= jb->n) break;
        int32_t b = a + chunk < jb->n ? a + chunk : jb->n;
        for (int32_t k = a; k < b; k += W16) {
            int nb = b - k < W16 ? b - k : W16;
            batch16(jb->p, jb->order + k, nb, jb->ref, jb->qer, jb->w, jb->maxsc, &sc);
        }
    }
    free(sc.s1); free(sc.s2); free(sc.H); free(sc.E);
    return NULL;
}

static int cmp_len(const void *a, const void *b)
{
    const SeqPair *x = *(SeqPair *const *)a, *y = *(SeqPair *const *)b;
    if (x->len2 != y->len2) return y->len2 - x->len2;
    return y->len1 - x->len1;
}

/* getScores16 equivalent on the host: sort by length (sortPairsLen), 8 pairs per SSE
 * batch, nthreads workers.  Pairs whose scores could overflow int16 or whose scoring
 * matrix is not match/mismatch/ambig form go through the scalar routine.  Returns 0. */
int sse41_get_scores16(const sse_params_t *p, SeqPair *pairs, const uint8_t *ref,
                       const uint8_t *qer, int32_t n, int32_t w, int nthreads)
{
    int maxsc = 0;
    for (int i = 0; i < 25; ++i) maxsc = maxsc > p->mat[i] ? maxsc : p->mat[i];
    int simple = 1;
    for (int t = 0; t < 5; ++t)
        for (int q = 0; q < 5; ++q) {
            int v = p->mat[t * 5 + q];
            int want = (t == 4 || q == 4) ? p->mat[4] : (t == q ? p->mat[0] : p->mat[1]);
            if (v != want) simple = 0;
        }
    SeqPair **order = (SeqPair **)malloc(sizeof(SeqPair *) * (n > 0 ? n : 1));
    int32_t m = 0;
    for (int32_t i = 0; i < n; ++i) {
        SeqPair *sp = &pairs[i];
        long hi = (long)sp->h0 + (long)maxsc * (sp->len1 < sp->len2 ? sp->len1 : sp->len2);
        if (!simple || hi > 32000 || sp->len1 > 32000 || sp->len2 > 32000) {
            sp->score = oracle_ksw_extend2(sp->len2, qer + sp->idq, sp->len1, ref + sp->idr, 5,
                                           p->mat, p->o_del, p->e_del, p->o_ins, p->e_ins, w,
                                           p->end_bonus, p->zdrop, sp->h0, &sp->qle, &sp->tle,
                                           &sp->gtle, &sp->gscore, &sp->max_off);
        } else {
            order[m++] = sp;
        }
    }
    qsort(order, (size_t)m, sizeof(SeqPair *), cmp_len);
    volatile int32_t next = 0;
    sse_job_t jb = {p, order, m, w, maxsc, ref, qer, &next};
    if (nthreads <= 1) {
        sse_worker(&jb);
    } else {
        pthread_t th[512];
        if (nthreads > 512) nthreads = 512;
        for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, sse_worker, &jb);
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    }
    free(order);
    return 0;
}
