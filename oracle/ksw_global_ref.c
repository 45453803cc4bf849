/*
 * ksw_global_ref.c -- TEST INFRASTRUCTURE (the CPU oracle of the global-alignment / CIGAR
 * batch).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it.
 *
 * A literal restatement of upstream's banded global alignment with traceback, ksw_global2 in
 * src/ksw.cpp (bwa's ksw.c; bwa-mem2 v2.2.1 keeps it unchanged) [UPSTREAM-RECALL, SURVEY.md
 * §2 row 3], as called from bwa_gen_cigar2 (src/bwa.cpp) for every final alignment of
 * mem_reg2aln.  No ksw.cpp ships in /root/reference: parity is unpinned by
 * reference fixtures and pinned instead by an independent matrix formulation in Python
 * (tests/ksw_global_py.py), hand-derived known answers and a CIGAR re-scoring property
 * (tests/test_global.py).
 *
 * Shape of the recurrence (target = rows i, query = columns j, band |i - j| <= w):
 *   first row : eh[0] = {0, -inf}, eh[j] = {-(o_ins + e_ins j), -inf} for 1 <= j <= min(qlen, w),
 *               {-inf, -inf} beyond
 *   row i     : beg = max(i - w, 0), end = min(i + w + 1, qlen),
 *               h1 = beg == 0 ? -(o_del + e_del (i + 1)) : -inf, f = -inf
 *   cell      : M = H(i-1,j-1) + S; H = max(M, E, F) with direction d = M >= E ? 0 : 1, then
 *               H >= F ? d : 2 (ties prefer M, then E); E' = max(E - e_del, M - oe_del) with bit
 *               (E - e_del > M - oe_del) << 2; F' = max(F - e_ins, M - oe_ins) with bit
 *               (F - e_ins > M - oe_ins) << 4 (upstream stores 2 << 4, read back as "2")
 *   row end   : eh[end] = {h1, -inf}
 *   score     : eh[qlen].h after the last row
 *   traceback : from (tlen - 1, min(tlen + w, qlen) - 1); state `which` = z >> (which << 1) & 3:
 *               0 -> M (--i, --k), 1 -> D (--i), 2 -> I (--k); then a leading D of i + 1 or
 *               I of k + 1; ops run-length merged (len << 4 | op, M = 0, I = 1, D = 2) and
 *               reversed.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define OG_MINUS_INF (-0x40000000)

typedef struct { int32_t h, e; } og_eh_t;

static uint32_t *og_push_cigar(int *n_cigar, int *m_cigar, uint32_t *cigar, int op, int len)
{
    if (*n_cigar == 0 || op != (int)(cigar[*n_cigar - 1] & 0xf)) {
        if (*n_cigar == *m_cigar) {
            *m_cigar = *m_cigar ? (*m_cigar) << 1 : 4;
            cigar = (uint32_t *)realloc(cigar, (size_t)(*m_cigar) * 4);
        }
        cigar[(*n_cigar)++] = (uint32_t)len << 4 | (uint32_t)op;
    } else
        cigar[*n_cigar - 1] += (uint32_t)len << 4;
    return cigar;
}

/* ksw_global2: returns the score; *n_cigar_ / *cigar_ (malloc'ed, caller frees) if non-null. */
int oracle_ksw_global2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
                       const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                       int *n_cigar_, uint32_t **cigar_)
{
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    const int want_cigar = n_cigar_ && cigar_;
    int i, j, k, score;
    if (n_cigar_) *n_cigar_ = 0;
    const int n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;      /* backtrack columns per row */
    uint8_t *z = want_cigar ? (uint8_t *)malloc((size_t)n_col * (size_t)tlen + 1) : 0;
    int8_t *qp = (int8_t *)malloc((size_t)qlen * m + 1);
    og_eh_t *eh = (og_eh_t *)calloc((size_t)qlen + 1, sizeof(og_eh_t));
    for (k = i = 0; k < m; ++k) {                                 /* query profile */
        const int8_t *p = &mat[k * m];
        for (j = 0; j < qlen; ++j) qp[i++] = p[query[j]];
    }
    eh[0].h = 0; eh[0].e = OG_MINUS_INF;                          /* first row */
    for (j = 1; j <= qlen && j <= w; ++j) eh[j].h = -(o_ins + e_ins * j), eh[j].e = OG_MINUS_INF;
    for (; j <= qlen; ++j) eh[j].h = eh[j].e = OG_MINUS_INF;
    for (i = 0; i < tlen; ++i) {
        int32_t f = OG_MINUS_INF, h1, beg, end, t;
        const int8_t *q = &qp[target[i] * qlen];
        beg = i > w ? i - w : 0;
        end = i + w + 1 < qlen ? i + w + 1 : qlen;
        h1 = beg == 0 ? -(o_del + e_del * (i + 1)) : OG_MINUS_INF;
        uint8_t *zi = want_cigar ? &z[(size_t)i * n_col] : 0;
        for (j = beg; j < end; ++j) {
            og_eh_t *p = &eh[j];
            int32_t h, mm = p->h, e = p->e;
            uint8_t d;
            p->h = h1;
            mm += q[j];
            d = mm >= e ? 0 : 1;
            h = mm >= e ? mm : e;
            d = h >= f ? d : 2;
            h = h >= f ? h : f;
            h1 = h;
            t = mm - oe_del;
            e -= e_del;
            d |= e > t ? 1 << 2 : 0;
            e = e > t ? e : t;
            p->e = e;
            t = mm - oe_ins;
            f -= e_ins;
            d |= f > t ? 2 << 4 : 0;
            f = f > t ? f : t;
            if (zi) zi[j - beg] = d;
        }
        eh[end].h = h1; eh[end].e = OG_MINUS_INF;
    }
    score = eh[qlen].h;
    if (want_cigar) {
        int n_cigar = 0, m_cigar = 0, which = 0;
        uint32_t *cigar = 0, tmp;
        i = tlen - 1; k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
        while (i >= 0 && k >= 0) {
            which = z[(size_t)i * n_col + (k - (i > w ? i - w : 0))] >> (which << 1) & 3;
            if (which == 0)      cigar = og_push_cigar(&n_cigar, &m_cigar, cigar, 0, 1), --i, --k;
            else if (which == 1) cigar = og_push_cigar(&n_cigar, &m_cigar, cigar, 2, 1), --i;
            else                 cigar = og_push_cigar(&n_cigar, &m_cigar, cigar, 1, 1), --k;
        }
        if (i >= 0) cigar = og_push_cigar(&n_cigar, &m_cigar, cigar, 2, i + 1);
        if (k >= 0) cigar = og_push_cigar(&n_cigar, &m_cigar, cigar, 1, k + 1);
        for (i = 0; i < n_cigar >> 1; ++i)
            tmp = cigar[i], cigar[i] = cigar[n_cigar - 1 - i], cigar[n_cigar - 1 - i] = tmp;
        *n_cigar_ = n_cigar, *cigar_ = cigar;
    }
    free(eh); free(qp); free(z);
    return score;
}

/* ------------------------------------------------------------------ batch form
 * Job i = pairs[i] (56-byte SeqPair, int32 fields idr, idq, id, len1, len2, h0, ...):
 * query = qer + idq (len2), target = ref + idr (len1), band w = h0.  score -> score[i];
 * CIGAR ops -> cigar[i * stride ...], count -> n_cigar[i]: -1 when more than `stride` ops,
 * -2 when qlen >= 1 and qlen < tlen - w (the traceback would start outside the band and
 * upstream reads outside the row's backtrack columns: not a defined result, and bwa_gen_cigar2
 * never asks for it since its w >= |tlen - qlen| + 3).  cigar == NULL: scores only. */
typedef struct { int32_t idr, idq, id, len1, len2, h0, seqid, regid, score, tle, gtle, qle, gscore, max_off; } og_pair_t;

typedef struct {
    const og_pair_t *pairs; const uint8_t *ref, *qer; int n;
    const int8_t *mat; int o_del, e_del, o_ins, e_ins;
    int32_t *score; uint32_t *cigar; int stride; int32_t *n_cigar;
    int t0, t1;
} og_job_t;

static void *og_worker(void *arg)
{
    og_job_t *J = (og_job_t *)arg;
    for (int i = J->t0; i < J->t1; ++i) {
        const og_pair_t *p = &J->pairs[i];
        const int bad = p->len2 >= 1 && p->len1 >= 1 && p->len2 < p->len1 - p->h0;
        const int tb = J->cigar && !bad;
        int nc = 0;
        uint32_t *cg = 0;
        J->score[i] = oracle_ksw_global2(p->len2, J->qer + p->idq, p->len1, J->ref + p->idr, 5, J->mat,
                                         J->o_del, J->e_del, J->o_ins, J->e_ins, p->h0,
                                         tb ? &nc : 0, tb ? &cg : 0);
        if (J->cigar) {
            if (bad)
                J->n_cigar[i] = -2;
            else if (nc <= J->stride) {
                if (nc) memcpy(J->cigar + (size_t)i * J->stride, cg, (size_t)nc * 4);
                J->n_cigar[i] = nc;
            } else
                J->n_cigar[i] = -1;
            free(cg);
        }
    }
    return 0;
}

void oracle_ksw_global2_batch(const void *pairs, const uint8_t *ref, const uint8_t *qer, int n,
                              const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins,
                              int32_t *score, uint32_t *cigar, int stride, int32_t *n_cigar, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 512) nthreads = 512;
    pthread_t th[512];
    og_job_t J[512];
    for (int t = 0; t < nthreads; ++t) {
        J[t] = (og_job_t){(const og_pair_t *)pairs, ref, qer, n, mat, o_del, e_del, o_ins, e_ins,
                          score, cigar, stride, n_cigar, (int)((int64_t)n * t / nthreads),
                          (int)((int64_t)n * (t + 1) / nthreads)};
        if (nthreads == 1) og_worker(&J[t]);
        else pthread_create(&th[t], 0, og_worker, &J[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], 0);
}
