/*
 * oracle/ksw_ext_ref.c -- CPU ORACLE (test infrastructure only).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline.  The product path
 * (bwa-mem2-arm_amd/csrc, libbsw_hip.so) never links or calls it.
 *
 * What it restates: scalar `ksw_extend2` from upstream bwa-mem2 v2.2.1 `src/ksw.cpp`
 * (= lh3/bwa ksw.c, bwa >= 0.7.11), which is also what upstream's
 * `BandedPairWiseSW::scalarBandedSWA` / `scalarBandedSWAWrapper` in `src/bandedSWA.cpp`
 * compute for each SeqPair.  The C++ of that fork is NOT vendored in /root/reference
 * (SURVEY.md §0.1-0.2); the algorithm is restated from SURVEY.md Appendix A (A.1-A.6),
 * the batch contract from SURVEY.md §3.2 / §8(c), and the reference's own call-site
 * evidence: ctor args docs-archive/INTEGRATION_COMPLETE.md:61-63, getScores signature
 * docs-archive/WEEK1_WRAPPER_COMPLETE.md:259-269, boundary rows / band cap
 * docs-archive/WEEK1_WRAPPER_COMPLETE.md:85-118.
 *
 * PARITY UNPINNED by the reference: /root/reference holds no golden vectors, no
 * fixtures and no test for this path, and its source cannot be
 * built here.  This oracle is pinned instead by (1) hand-derived known-answer tests
 * (tests/test_oracle.py), (2) two independent transcriptions: the line-by-line Python one
 * (oracle/ksw_ext_ref.py, small pairs in tests/test_oracle.py) and the vectorised numpy one
 * (oracle/ksw_ext_np.py: every committed golden pair in tests/test_oracle.py, and 10^6 C2
 * pairs + 4 x 10^5 pairs of other classes in tests/oracle_crosscheck.py, recorded output
 * tests/golden/crosscheck_1e6.json), and (3) the committed golden fixtures in tests/golden/
 * generated from it (tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../include/bsw_seqpair.h"

typedef struct { int32_t h, e; } eh_t;

/* ksw_extend2 (Appendix A).  Row i walks the target (ref, len1), column j the query
 * (len2).  Returns the best score; out-params as upstream. */
/* Band cells the literal loop visits (sum of end - beg over rows), per thread: the "actual cells"
 * of SURVEY.md §8(d), read by bench.py on a sample. */
static __thread long long g_oracle_cells;
long long oracle_cells_take(void)
{
    const long long c = g_oracle_cells;
    g_oracle_cells = 0;
    return c;
}

int oracle_ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target,
                       int m, const int8_t *mat, int o_del, int e_del, int o_ins,
                       int e_ins, int w, int end_bonus, int zdrop, int h0, int *_qle,
                       int *_tle, int *_gtle, int *_gscore, int *_max_off)
{
    eh_t *eh;
    int8_t *qp;
    int i, j, k, oe_del = o_del + e_del, oe_ins = o_ins + e_ins, beg, end, max, max_i,
        max_j, max_ins, max_del, max_ie, gscore, max_off;

    /* query profile qp[t*qlen + j] = mat[t*m + query[j]] */
    qp = (int8_t *)malloc((size_t)(qlen > 0 ? qlen : 1) * m);
    /* A.1: upstream allocates qlen+1 entries and still writes eh[1] when qlen == 0;
     * one spare entry keeps that write in bounds without changing any read. */
    eh = (eh_t *)calloc((size_t)qlen + 2, sizeof(eh_t));
    for (k = i = 0; k < m; ++k) {
        const int8_t *p = &mat[k * m];
        for (j = 0; j < qlen; ++j) qp[i++] = p[query[j]];
    }
    /* A.1 first row */
    eh[0].h = h0;
    eh[1].h = h0 > oe_ins ? h0 - oe_ins : 0;
    for (j = 2; j <= qlen && eh[j - 1].h > e_ins; ++j) eh[j].h = eh[j - 1].h - e_ins;
    /* A.2 band cap */
    k = m * m;
    for (i = 0, max = 0; i < k; ++i) max = max > mat[i] ? max : mat[i];
    max_ins = (int)((double)(qlen * max + end_bonus - o_ins) / e_ins + 1.);
    max_ins = max_ins > 1 ? max_ins : 1;
    w = w < max_ins ? w : max_ins;
    max_del = (int)((double)(qlen * max + end_bonus - o_del) / e_del + 1.);
    max_del = max_del > 1 ? max_del : 1;
    w = w < max_del ? w : max_del;
    /* A.3 */
    max = h0, max_i = max_j = -1;
    max_ie = -1, gscore = -1;
    max_off = 0;
    beg = 0, end = qlen;
    /* A.4 */
    for (i = 0; i < tlen; ++i) {
        int t, f = 0, h1, mm = 0, mj = -1;
        int8_t *q = &qp[target[i] * qlen];
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        if (beg == 0) {
            h1 = h0 - (o_del + e_del * (i + 1));
            if (h1 < 0) h1 = 0;
        } else
            h1 = 0;
        if (end > beg) g_oracle_cells += end - beg;
        for (j = beg; j < end; ++j) {
            /* eh[j] = { H(i-1,j-1), E(i,j) }, f = F(i,j), h1 = H(i,j-1) */
            eh_t *p = &eh[j];
            int h, M = p->h, e = p->e;
            p->h = h1;
            M = M ? M + q[j] : 0;
            h = M > e ? M : e;
            h = h > f ? h : f;
            h1 = h;
            mj = mm > h ? mj : j;
            mm = mm > h ? mm : h;
            t = M - oe_del;
            t = t > 0 ? t : 0;
            e -= e_del;
            e = e > t ? e : t;
            p->e = e;
            t = M - oe_ins;
            t = t > 0 ? t : 0;
            f -= e_ins;
            f = f > t ? f : t;
        }
        eh[end].h = h1;
        eh[end].e = 0;
        if (j == qlen) {
            max_ie = gscore > h1 ? max_ie : i;
            gscore = gscore > h1 ? gscore : h1;
        }
        if (mm == 0) break;
        if (mm > max) {
            max = mm, max_i = i, max_j = mj;
            max_off = max_off > abs(mj - i) ? max_off : abs(mj - i);
        } else if (zdrop > 0) {
            if (i - max_i > mj - max_j) {
                if (max - mm - ((i - max_i) - (mj - max_j)) * e_del > zdrop) break;
            } else {
                if (max - mm - ((mj - max_j) - (i - max_i)) * e_ins > zdrop) break;
            }
        }
        /* A.4 narrowing */
        for (j = beg; j < end && eh[j].h == 0 && eh[j].e == 0; ++j)
            ;
        beg = j;
        for (j = end; j >= beg && eh[j].h == 0 && eh[j].e == 0; --j)
            ;
        end = j + 2 < qlen ? j + 2 : qlen;
    }
    free(eh);
    free(qp);
    if (_qle) *_qle = max_j + 1;
    if (_tle) *_tle = max_i + 1;
    if (_gtle) *_gtle = max_ie + 1;
    if (_gscore) *_gscore = gscore;
    if (_max_off) *_max_off = max_off;
    return max;
}

/* The scoring parameters the batch entry points take (mirror of bsw_params_t). */
typedef struct {
    int32_t o_del, e_del, o_ins, e_ins, zdrop, end_bonus;
    int8_t mat[25];
} oracle_params_t;

/* scalarBandedSWAWrapper: for each pair, seq1 = ref (len1, rows), seq2 = query
 * (len2, columns); outputs written in place.  [UPSTREAM-RECALL, SURVEY.md §3.3] */
void oracle_get_scores(const oracle_params_t *p, SeqPair *pairs, const uint8_t *seqBufRef,
                       const uint8_t *seqBufQer, int32_t n, int32_t w)
{
    for (int32_t i = 0; i < n; ++i) {
        SeqPair *sp = &pairs[i];
        sp->score = oracle_ksw_extend2(sp->len2, seqBufQer + sp->idq, sp->len1,
                                       seqBufRef + sp->idr, 5, p->mat, p->o_del, p->e_del,
                                       p->o_ins, p->e_ins, w, p->end_bonus, p->zdrop, sp->h0,
                                       &sp->qle, &sp->tle, &sp->gtle, &sp->gscore,
                                       &sp->max_off);
    }
}

/* Multi-threaded form for the CPU-baseline leg (pthreads, contiguous ranges). */
#include <pthread.h>
typedef struct {
    const oracle_params_t *p;
    SeqPair *pairs;
    const uint8_t *r, *q;
    int32_t n, w;
} oracle_job_t;
static void *oracle_worker(void *arg)
{
    oracle_job_t *j = (oracle_job_t *)arg;
    oracle_get_scores(j->p, j->pairs, j->r, j->q, j->n, j->w);
    return NULL;
}
void oracle_get_scores_mt(const oracle_params_t *p, SeqPair *pairs, const uint8_t *r,
                          const uint8_t *q, int32_t n, int32_t w, int nthreads)
{
    if (nthreads <= 1 || n < 2 * nthreads) {
        oracle_get_scores(p, pairs, r, q, n, w);
        return;
    }
    pthread_t th[512];
    oracle_job_t jobs[512];
    if (nthreads > 512) nthreads = 512;
    for (int t = 0; t < nthreads; ++t) {
        int32_t a = (int32_t)((int64_t)n * t / nthreads), b = (int32_t)((int64_t)n * (t + 1) / nthreads);
        jobs[t] = (oracle_job_t){p, pairs + a, r, q, b - a, w};
        pthread_create(&th[t], NULL, oracle_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}
