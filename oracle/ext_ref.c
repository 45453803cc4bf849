/*
 * ext_ref.c -- CPU restatement of the seed-extension consumer (TEST INFRASTRUCTURE ONLY: the
 * checker for bwa-mem2-arm_amd/csrc/bsw_ext.cpp; never linked into the product).
 *
 * Literal per-read form of the extension half of upstream mem_chain2aln (bwa 0.7.x
 * src/bwamem.c, which bwa-mem2's src/bwamem.cpp keeps; [UPSTREAM-RECALL], SURVEY.md a9 /
 * §8(f) row 1), one seed per read: target window via cal_max_gap, LEFT extension on reversed
 * sequences with h0 = seed score and the MAX_BAND_TRY loop, local vs to-end by pen_clip5,
 * RIGHT extension with h0 = the LEFT score, pen_clip3.  Scoring through oracle_ksw_extend2.
 * Parity unpinned by the reference (no upstream fixtures for this step), like the oracle.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../include/bsw_ext.h"

int oracle_ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
                       const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                       int end_bonus, int zdrop, int h0, int *_qle, int *_tle, int *_gtle,
                       int *_gscore, int *_max_off);

typedef struct {
    int32_t o_del, e_del, o_ins, e_ins, zdrop, end_bonus;
    int8_t mat[25];
} oracle_params_t;

static int cal_max_gap(const oracle_params_t *p, int a, int w, int qlen)
{
    int l_del = (int)((double)(qlen * a - p->o_del) / p->e_del + 1.);
    int l_ins = (int)((double)(qlen * a - p->o_ins) / p->e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < w << 1 ? l : w << 1;
}

/* mem_chain2aln's target window over seeds[0, n) of one chain (bwa 0.7.x src/bwamem.c, the rmax[]
 * loop at the top of mem_chain2aln): min / max over the seeds of the per-seed reach, clipped to
 * [0, ref_len); with l_pac > 0 (ref = forward + reverse-complement text) a window crossing l_pac
 * keeps the side of the chain's first seed.  Seeds with len <= 0 (no seed) take no part. */
void oracle_chain_window(const oracle_params_t *p, const bsw_ext_opt_t *opt, int64_t ref_len, int l_query,
                         const bsw_seed_t *const *seeds, int n, int64_t *rmax0, int64_t *rmax1)
{
    const int a = p->mat[0];
    int64_t lo = ref_len, hi = 0, first = -1;
    for (int i = 0; i < n; ++i) {
        const bsw_seed_t *t = seeds[i];
        if (t->len <= 0) continue;
        if (first < 0) first = t->rbeg;
        const int64_t b = t->rbeg - (t->qbeg + cal_max_gap(p, a, opt->w, t->qbeg));
        const int64_t e = t->rbeg + t->len + ((l_query - t->qbeg - t->len) +
                                              cal_max_gap(p, a, opt->w, l_query - t->qbeg - t->len));
        lo = lo < b ? lo : b;
        hi = hi > e ? hi : e;
    }
    lo = lo > 0 ? lo : 0;
    hi = hi < ref_len ? hi : ref_len;
    if (opt->l_pac > 0 && lo < opt->l_pac && opt->l_pac < hi) {   /* crossing the forward-reverse boundary */
        if (first < opt->l_pac) hi = opt->l_pac;
        else lo = opt->l_pac;
    }
    *rmax0 = lo;
    *rmax1 = hi;
}

/* one seed's extension inside the window [rmax0, rmax1) (the body of mem_chain2aln's per-seed step) */
static void oracle_extend_one(const oracle_params_t *p, const bsw_ext_opt_t *opt, const uint8_t *ref,
                              int64_t rmax0, int64_t rmax1, const uint8_t *query, int l_query,
                              const bsw_seed_t *s, bsw_alnreg_t *r)
{
    const int a = p->mat[0];
    {
        int qle, tle, gtle, gscore, max_off[2] = {0, 0}, aw[2];
        memset(r, 0, sizeof(*r));
        if (s->len <= 0) return;
        aw[0] = aw[1] = opt->w;
        r->score = r->truesc = -1;                       /* as upstream: the first try's prev */
        r->seedlen0 = s->len;
        if (s->qbeg) {                                   /* left extension */
            int tmp = (int)(s->rbeg - rmax0);
            uint8_t *qs = (uint8_t *)malloc((size_t)s->qbeg), *rs = (uint8_t *)malloc((size_t)(tmp > 0 ? tmp : 1));
            for (int k = 0; k < s->qbeg; ++k) qs[k] = query[s->qbeg - 1 - k];
            for (int k = 0; k < tmp; ++k) rs[k] = ref[s->rbeg - 1 - k];
            for (int t = 0; t < opt->max_band_try; ++t) {
                int prev = r->score;
                aw[0] = opt->w << t;
                r->score = oracle_ksw_extend2(s->qbeg, qs, tmp, rs, 5, p->mat, p->o_del, p->e_del, p->o_ins,
                                              p->e_ins, aw[0], opt->pen_clip5, p->zdrop, s->len * a, &qle,
                                              &tle, &gtle, &gscore, &max_off[0]);
                if (r->score == prev || max_off[0] < (aw[0] >> 1) + (aw[0] >> 2)) break;
            }
            if (gscore <= 0 || gscore <= r->score - opt->pen_clip5) {   /* local */
                r->qb = s->qbeg - qle; r->rb = s->rbeg - tle;
                r->truesc = r->score;
            } else {                                                    /* to-end */
                r->qb = 0; r->rb = s->rbeg - gtle;
                r->truesc = gscore;
            }
            free(qs); free(rs);
        } else {
            r->score = r->truesc = s->len * a; r->qb = 0; r->rb = s->rbeg;
        }
        if (s->qbeg + s->len != l_query) {               /* right extension */
            int qe = s->qbeg + s->len;
            int64_t re = s->rbeg + s->len;
            int sc0 = r->score;
            for (int t = 0; t < opt->max_band_try; ++t) {
                int prev = r->score;
                aw[1] = opt->w << t;
                r->score = oracle_ksw_extend2(l_query - qe, query + qe, (int)(rmax1 - re), ref + re, 5, p->mat,
                                              p->o_del, p->e_del, p->o_ins, p->e_ins, aw[1], opt->pen_clip3,
                                              p->zdrop, sc0, &qle, &tle, &gtle, &gscore, &max_off[1]);
                if (r->score == prev || max_off[1] < (aw[1] >> 1) + (aw[1] >> 2)) break;
            }
            if (gscore <= 0 || gscore <= r->score - opt->pen_clip3) {   /* local */
                r->qe = qe + qle; r->re = re + tle;
                r->truesc += r->score - sc0;
            } else {                                                    /* to-end */
                r->qe = l_query; r->re = re + gtle;
                r->truesc += gscore - sc0;
            }
        } else {
            r->qe = l_query; r->re = s->rbeg + s->len;
        }
        r->w = aw[0] > aw[1] ? aw[0] : aw[1];
    }
}

void oracle_extend_seeds(const oracle_params_t *p, const bsw_ext_opt_t *opt, const uint8_t *ref,
                         int64_t ref_len, const uint8_t *reads, const int64_t *read_off,
                         const int32_t *read_len, const bsw_seed_t *seeds, int32_t n,
                         bsw_alnreg_t *out)
{
    for (int32_t i = 0; i < n; ++i) {                   /* every seed a chain of one */
        const bsw_seed_t *s = &seeds[i];
        int64_t r0 = 0, r1 = 0;
        oracle_chain_window(p, opt, ref_len, read_len[i], &s, 1, &r0, &r1);
        oracle_extend_one(p, opt, ref, r0, r1, reads + read_off[i], read_len[i], s, &out[i]);
    }
}

/* mem_chain2aln over the chains of every read, literal per-read order (bwa 0.7.x src/bwamem.c,
 * kept by bwa-mem2's src/bwamem.cpp; [UPSTREAM-RECALL]): the read's
 * chains in the given order, each chain's seeds by score descending (ties: the later seed
 * first, bwa's srt[] = score << 32 | index sorted ascending and walked down); a seed is
 * skipped when an earlier region of the READ (any chain) contains it "around" the same
 * diagonal -- unless an extended, at least 95%-as-long seed of its own chain overlaps it on a
 * different diagonal; otherwise it is extended (oracle_extend_one) and its region appended.
 * Seeds are grouped by read (seed_read non-decreasing), chains are runs of equal seed_chain; every
 * seed of a chain extends inside the chain's one target window (oracle_chain_window). */
static int oracle_contained(const oracle_params_t *p, const bsw_ext_opt_t *opt, const bsw_seed_t *s,
                            int l_query, const bsw_alnreg_t *out, const int32_t *av, int nav)
{
    const int a = p->mat[0];
    for (int i = 0; i < nav; ++i) {
        const bsw_alnreg_t *q = &out[av[i]];
        int64_t rd;
        int qd, w, max_gap;
        if (s->rbeg < q->rb || s->rbeg + s->len > q->re || s->qbeg < q->qb || s->qbeg + s->len > q->qe) continue;
        if (s->len - q->seedlen0 > .1 * l_query) continue;
        qd = s->qbeg - q->qb; rd = s->rbeg - q->rb;
        max_gap = cal_max_gap(p, a, opt->w, qd < rd ? qd : (int)rd);
        w = max_gap < q->w ? max_gap : q->w;
        if (qd - rd < w && rd - qd < w) return 1;
        qd = q->qe - (s->qbeg + s->len); rd = q->re - (s->rbeg + s->len);
        max_gap = cal_max_gap(p, a, opt->w, qd < rd ? qd : (int)rd);
        w = max_gap < q->w ? max_gap : q->w;
        if (qd - rd < w && rd - qd < w) return 1;
    }
    return 0;
}

void oracle_chain2aln(const oracle_params_t *p, const bsw_ext_opt_t *opt, const uint8_t *ref, int64_t ref_len,
                      const uint8_t *reads, const int64_t *read_off, const int32_t *read_len,
                      const bsw_seed_t *seeds, const int32_t *seed_read, const int32_t *seed_chain, int32_t ns,
                      bsw_alnreg_t *out, int32_t *extended)
{
    const int a = p->mat[0];
    int32_t *av = (int32_t *)malloc(sizeof(int32_t) * (size_t)(ns > 0 ? ns : 1));
    int32_t *srt = (int32_t *)malloc(sizeof(int32_t) * (size_t)(ns > 0 ? ns : 1));
    for (int32_t k = 0; k < ns; ++k) { memset(&out[k], 0, sizeof(out[k])); extended[k] = 0; }
    for (int32_t r0 = 0; r0 < ns;) {
        int32_t r1 = r0;
        while (r1 < ns && seed_read[r1] == seed_read[r0]) ++r1;
        const int rid = seed_read[r0];
        const uint8_t *query = reads + read_off[rid];
        const int l_query = read_len[rid];
        int nav = 0;
        for (int32_t c0 = r0; c0 < r1;) {
            int32_t c1 = c0;
            while (c1 < r1 && seed_chain[c1] == seed_chain[c0]) ++c1;
            const int n = c1 - c0;
            int64_t rmax0 = 0, rmax1 = 0;                   /* the chain's target window */
            {
                const bsw_seed_t **cs = (const bsw_seed_t **)malloc(sizeof(*cs) * (size_t)n);
                for (int i = 0; i < n; ++i) cs[i] = &seeds[c0 + i];
                oracle_chain_window(p, opt, ref_len, l_query, cs, n, &rmax0, &rmax1);
                free(cs);
            }
            /* srt ascending by (score, index); processed from the top down */
            for (int i = 0; i < n; ++i) srt[i] = c0 + i;
            for (int i = 1; i < n; ++i)
                for (int j = i; j > 0; --j) {
                    const int32_t x = srt[j - 1], y = srt[j];
                    const int64_t kx = ((int64_t)(seeds[x].len * a) << 32) | (x - c0);
                    const int64_t ky = ((int64_t)(seeds[y].len * a) << 32) | (y - c0);
                    if (kx > ky) { srt[j - 1] = y; srt[j] = x; } else break;
                }
            for (int k = n - 1; k >= 0; --k) {
                const int32_t si = srt[k];
                const bsw_seed_t *s = &seeds[si];
                if (oracle_contained(p, opt, s, l_query, out, av, nav)) {
                    int i;
                    for (i = k + 1; i < n; ++i) {          /* overlapping extended seeds of the chain */
                        const bsw_seed_t *t;
                        if (!extended[srt[i]]) continue;
                        t = &seeds[srt[i]];
                        if (t->len < s->len * .95) continue;
                        if (s->qbeg <= t->qbeg && s->qbeg + s->len - t->qbeg >= s->len >> 2 &&
                            t->qbeg - s->qbeg != t->rbeg - s->rbeg) break;
                        if (t->qbeg <= s->qbeg && t->qbeg + t->len - s->qbeg >= s->len >> 2 &&
                            s->qbeg - t->qbeg != s->rbeg - t->rbeg) break;
                    }
                    if (i == n) continue;                   /* skipped: not extended */
                }
                oracle_extend_one(p, opt, ref, rmax0, rmax1, query, l_query, s, &out[si]);
                extended[si] = 1;
                av[nav++] = si;
            }
            c0 = c1;
        }
        r0 = r1;
    }
    free(av);
    free(srt);
}

/* oracle_chain2aln over nthreads pthreads, reads split into contiguous runs (reads are
 * independent; the bench's multi-thread CPU baseline leg). */
#include <pthread.h>
typedef struct {
    const oracle_params_t *p;
    const bsw_ext_opt_t *opt;
    const uint8_t *ref, *reads;
    int64_t ref_len;
    const int64_t *read_off;
    const int32_t *read_len;
    const bsw_seed_t *seeds;
    const int32_t *seed_read, *seed_chain;
    int32_t a, b;
    bsw_alnreg_t *out;
    int32_t *extended;
} c2a_job_t;

static void *c2a_worker(void *arg)
{
    c2a_job_t *j = (c2a_job_t *)arg;
    oracle_chain2aln(j->p, j->opt, j->ref, j->ref_len, j->reads, j->read_off, j->read_len, j->seeds + j->a,
                     j->seed_read + j->a, j->seed_chain + j->a, j->b - j->a, j->out + j->a, j->extended + j->a);
    return NULL;
}

void oracle_chain2aln_mt(const oracle_params_t *p, const bsw_ext_opt_t *opt, const uint8_t *ref, int64_t ref_len,
                         const uint8_t *reads, const int64_t *read_off, const int32_t *read_len,
                         const bsw_seed_t *seeds, const int32_t *seed_read, const int32_t *seed_chain, int32_t ns,
                         bsw_alnreg_t *out, int32_t *extended, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    c2a_job_t jobs[256];
    int32_t a = 0;
    for (int t = 0; t < nthreads; ++t) {
        int32_t b = (int32_t)((int64_t)ns * (t + 1) / nthreads);
        while (b > a && b < ns && seed_read[b] == seed_read[b - 1]) ++b;     /* whole reads per thread */
        if (b < a) b = a;
        c2a_job_t j = {p, opt, ref, reads, ref_len, read_off, read_len, seeds, seed_read, seed_chain, a, b, out,
                       extended};
        jobs[t] = j;
        a = b;
    }
    jobs[nthreads - 1].b = ns;
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, c2a_worker, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}
