/*
 * chain_ref.c -- CPU restatement of bwa's seed chaining (TEST INFRASTRUCTURE ONLY: the checker
 * for bwa-mem2-arm_amd/csrc/bsw_memchain.hip; never linked into the product).
 *
 * Literal per-read transcription of mem_chain, test_and_merge, mem_chain_weight and
 * mem_chain_flt (lh3/bwa src/bwamem.c 0.7.17, which bwa-mem2 v2.2.1's src/bwamem.cpp keeps;
 * [UPSTREAM-RECALL]: /root/reference holds no source of them), with klib's
 * ks_introsort / ks_combsort / insertion sort (ksort.h) for mem_chain_flt's weight sort and a
 * sorted array standing in for the kbtree of chains (kb_intervalp = the first chain of equal
 * start, else the last chain of smaller start; a new chain goes right after the first chain
 * of equal start: what a single-leaf kbtree does).  Parity unpinned by the reference.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../include/bsw_fmi.h"

typedef struct {
    int64_t rbeg;
    int32_t qbeg, len, score;
} oseed_t;

typedef struct {
    int n, m;
    int64_t pos;
    oseed_t *seeds;
    int w, kept, first;
} ochain_t;

/* test_and_merge (bwamem.c): 1 if seed p was absorbed by chain c (or is contained in it) */
static int test_and_merge(const bsw_chain_opt_t *opt, int64_t l_pac, ochain_t *c, const oseed_t *p)
{
    int64_t qend, rend, x, y;
    const oseed_t *last = &c->seeds[c->n - 1];
    qend = last->qbeg + last->len;
    rend = last->rbeg + last->len;
    /* one contig: seed_rid == c->rid always */
    if (p->qbeg >= c->seeds[0].qbeg && p->qbeg + p->len <= qend && p->rbeg >= c->seeds[0].rbeg &&
        p->rbeg + p->len <= rend)
        return 1;                                     /* contained seed; do nothing */
    if ((last->rbeg < l_pac || c->seeds[0].rbeg < l_pac) && p->rbeg >= l_pac) return 0;   /* other strand */
    x = p->qbeg - last->qbeg;
    y = p->rbeg - last->rbeg;
    if (y >= 0 && x - y <= opt->w && y - x <= opt->w && x - last->len < opt->max_chain_gap &&
        y - last->len < opt->max_chain_gap) {       /* grow the chain */
        if (c->n == c->m) {
            c->m <<= 1;
            c->seeds = (oseed_t *)realloc(c->seeds, (size_t)c->m * sizeof(oseed_t));
        }
        c->seeds[c->n++] = *p;
        return 1;
    }
    return 0;
}

static int chain_weight(const ochain_t *c)
{
    int64_t end;
    int j, w = 0, tmp;
    for (j = 0, end = 0; j < c->n; ++j) {
        const oseed_t *s = &c->seeds[j];
        if (s->qbeg >= end) w += s->len;
        else if (s->qbeg + s->len > end) w += (int)(s->qbeg + s->len - end);
        end = end > s->qbeg + s->len ? end : s->qbeg + s->len;
    }
    tmp = w; w = 0;
    for (j = 0, end = 0; j < c->n; ++j) {
        const oseed_t *s = &c->seeds[j];
        if (s->rbeg >= end) w += s->len;
        else if (s->rbeg + s->len > end) w += (int)(s->rbeg + s->len - end);
        end = end > s->rbeg + s->len ? end : s->rbeg + s->len;
    }
    w = w < tmp ? w : tmp;
    return w < 1 << 30 ? w : (1 << 30) - 1;
}

/* ---- klib ksort.h, instantiated for ochain_t with flt_lt(a, b) = a.w > b.w */
#define flt_lt(a, b) ((a).w > (b).w)

static void insertsort_flt(ochain_t *s, ochain_t *t)
{
    ochain_t *i, *j, swap_tmp;
    for (i = s + 1; i < t; ++i)
        for (j = i; j > s && flt_lt(*j, *(j - 1)); --j) {
            swap_tmp = *j; *j = *(j - 1); *(j - 1) = swap_tmp;
        }
}

static void combsort_flt(size_t n, ochain_t a[])
{
    const double shrink_factor = 1.2473309501039786540366528676643;
    int do_swap;
    size_t gap = n;
    ochain_t tmp, *i, *j;
    do {
        if (gap > 2) {
            gap = (size_t)(gap / shrink_factor);
            if (gap == 9 || gap == 10) gap = 11;
        }
        do_swap = 0;
        for (i = a; i < a + n - gap; ++i) {
            j = i + gap;
            if (flt_lt(*j, *i)) {
                tmp = *i; *i = *j; *j = tmp;
                do_swap = 1;
            }
        }
    } while (do_swap || gap > 2);
    if (gap != 1) insertsort_flt(a, a + n);
}

typedef struct { ochain_t *left, *right; int depth; } isort_stack_t;

static void introsort_flt(size_t n, ochain_t a[])
{
    int d;
    isort_stack_t *top, *stack;
    ochain_t rp, swap_tmp;
    ochain_t *s, *t, *i, *j, *k;
    if (n < 1) return;
    else if (n == 2) {
        if (flt_lt(a[1], a[0])) { swap_tmp = a[0]; a[0] = a[1]; a[1] = swap_tmp; }
        return;
    }
    for (d = 2; 1ul << d < n; ++d) ;
    stack = (isort_stack_t *)malloc(sizeof(isort_stack_t) * ((sizeof(size_t) * d) + 2));
    top = stack; s = a; t = a + (n - 1); d <<= 1;
    while (1) {
        if (s < t) {
            if (--d == 0) {
                combsort_flt((size_t)(t - s + 1), s);
                t = s;
                continue;
            }
            i = s; j = t; k = i + ((j - i) >> 1) + 1;
            if (flt_lt(*k, *i)) {
                if (flt_lt(*k, *j)) k = j;
            } else k = flt_lt(*j, *i) ? i : j;
            rp = *k;
            if (k != t) { swap_tmp = *k; *k = *t; *t = swap_tmp; }
            for (;;) {
                do ++i; while (flt_lt(*i, rp));
                do --j; while (i <= j && flt_lt(rp, *j));
                if (j <= i) break;
                swap_tmp = *i; *i = *j; *j = swap_tmp;
            }
            swap_tmp = *i; *i = *t; *t = swap_tmp;
            if (i - s > t - i) {
                if (i - s > 16) { top->left = s; top->right = i - 1; top->depth = d; ++top; }
                s = t - i > 16 ? i + 1 : t;
            } else {
                if (t - i > 16) { top->left = i + 1; top->right = t; top->depth = d; ++top; }
                t = i - s > 16 ? i - 1 : s;
            }
        } else {
            if (top == stack) {
                free(stack);
                insertsort_flt(a, a + n);
                return;
            } else {
                --top; s = top->left; t = top->right; d = top->depth;
            }
        }
    }
}

#define chn_beg(ch) ((ch).seeds->qbeg)
#define chn_end(ch) ((ch).seeds[(ch).n - 1].qbeg + (ch).seeds[(ch).n - 1].len)

/* mem_chain_flt (bwamem.c): returns the number of chains kept, a[0 .. k) */
static int chain_flt(const bsw_chain_opt_t *opt, int n_chn, ochain_t *a)
{
    int i, k, nch = 0;
    int *chains;
    if (n_chn == 0) return 0;
    for (i = k = 0; i < n_chn; ++i) {
        ochain_t *c = &a[i];
        c->first = -1; c->kept = 0;
        c->w = chain_weight(c);
        if (c->w < opt->min_chain_weight) free(c->seeds);
        else a[k++] = *c;
    }
    n_chn = k;
    if (n_chn == 0) return 0;
    introsort_flt((size_t)n_chn, a);
    chains = (int *)malloc(sizeof(int) * (size_t)n_chn);
    a[0].kept = 3;
    chains[nch++] = 0;
    for (i = 1; i < n_chn; ++i) {
        int large_ovlp = 0;
        for (k = 0; k < nch; ++k) {
            int j = chains[k];
            int b_max = chn_beg(a[j]) > chn_beg(a[i]) ? chn_beg(a[j]) : chn_beg(a[i]);
            int e_min = chn_end(a[j]) < chn_end(a[i]) ? chn_end(a[j]) : chn_end(a[i]);
            if (e_min > b_max) {                      /* no ALT contigs: is_alt == 0 everywhere */
                int li = chn_end(a[i]) - chn_beg(a[i]);
                int lj = chn_end(a[j]) - chn_beg(a[j]);
                int min_l = li < lj ? li : lj;
                if (e_min - b_max >= min_l * opt->mask_level && min_l < opt->max_chain_gap) {
                    large_ovlp = 1;
                    if (a[j].first < 0) a[j].first = i;
                    if (a[i].w < a[j].w * opt->drop_ratio && a[j].w - a[i].w >= opt->min_seed_len << 1) break;
                }
            }
        }
        if (k == nch) {
            chains[nch++] = i;
            a[i].kept = large_ovlp ? 2 : 3;
        }
    }
    for (i = 0; i < nch; ++i) {
        ochain_t *c = &a[chains[i]];
        if (c->first >= 0) a[c->first].kept = 1;
    }
    free(chains);
    for (i = k = 0; i < n_chn; ++i) {
        if (a[i].kept == 0 || a[i].kept == 3) continue;
        if (++k >= opt->max_chain_extend) break;
    }
    for (; i < n_chn; ++i)
        if (a[i].kept < 3) a[i].kept = 0;
    for (i = k = 0; i < n_chn; ++i) {
        ochain_t *c = &a[i];
        if (c->kept == 0) free(c->seeds);
        else a[k++] = a[i];
    }
    return k;
}

/* mem_chain for one read: chains in start order (the kbtree traversal) */
/* SA lookups: a plain array, or an FM-index's bwt_sa (oracle_fmi_sa_at: the lean index's LF walks) */
typedef struct { const int64_t *sa; const void *fmi; } sa_src_t;
int64_t oracle_fmi_sa_at(const void *f, int64_t r);
static int64_t sa_get(const sa_src_t *s, int64_t r) { return s->fmi ? oracle_fmi_sa_at(s->fmi, r) : s->sa[r]; }

static int read_chains(const bsw_chain_opt_t *opt, const sa_src_t *sa, int64_t l_pac, int len,
                       const bsw_bwtintv_t *mem, int n_mem, ochain_t **out)
{
    int n = 0, m = 16;
    ochain_t *a = (ochain_t *)malloc(sizeof(ochain_t) * (size_t)m);
    *out = a;
    if (len < opt->min_seed_len) return 0;
    for (int i = 0; i < n_mem; ++i) {
        const bsw_bwtintv_t *p = &mem[i];
        const int slen = (int)((uint32_t)p->info - (p->info >> 32));
        const int64_t step = (int64_t)p->x[2] > opt->max_occ ? (int64_t)p->x[2] / opt->max_occ : 1;
        int64_t k;
        int count;
        for (k = count = 0; k < (int64_t)p->x[2] && count < opt->max_occ; k += step, ++count) {
            oseed_t s;
            s.rbeg = sa_get(sa, (int64_t)p->x[0] + k);
            s.qbeg = (int32_t)(p->info >> 32);
            s.score = s.len = slen;
            if (s.rbeg < l_pac && l_pac < s.rbeg + s.len) continue;   /* bns_intv2rid < 0: bridging */
            /* kb_intervalp: lower = first chain with pos == rbeg, else last with pos < rbeg */
            int lo = 0, hi = n;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (a[mid].pos < s.rbeg) lo = mid + 1; else hi = mid;
            }
            const int eq = lo < n && a[lo].pos == s.rbeg;
            const int lower = eq ? lo : lo - 1;
            if (lower >= 0 && test_and_merge(opt, l_pac, &a[lower], &s)) continue;
            const int at = eq ? lo + 1 : lo;                          /* kb_putp position */
            if (n == m) {
                m <<= 1;
                a = (ochain_t *)realloc(a, sizeof(ochain_t) * (size_t)m);
                *out = a;
            }
            memmove(&a[at + 1], &a[at], sizeof(ochain_t) * (size_t)(n - at));
            ochain_t *c = &a[at];
            memset(c, 0, sizeof(*c));
            c->n = 1; c->m = 4;
            c->seeds = (oseed_t *)calloc((size_t)c->m, sizeof(oseed_t));
            c->seeds[0] = s;
            c->pos = s.rbeg;
            ++n;
        }
    }
    return n;
}

/* Every read: mem_chain + mem_chain_flt -> seeds grouped by read / chain (bsw_fmi.h's output
 * layout).  Returns the number of seeds (written only while < seed_cap). */
static int64_t mem_chain_src(const bsw_chain_opt_t *opt, const sa_src_t *sa, int64_t l_pac, const int32_t *read_len,
                             int32_t n_reads, const bsw_bwtintv_t *mems, int32_t cap, const int32_t *n_mems,
                             bsw_seed_t *seeds, int32_t *seed_read, int32_t *seed_chain, int64_t seed_cap);
int64_t oracle_mem_chain(const bsw_chain_opt_t *opt, const int64_t *sa, int64_t l_pac, const int32_t *read_len,
                         int32_t n_reads, const bsw_bwtintv_t *mems, int32_t cap, const int32_t *n_mems,
                         bsw_seed_t *seeds, int32_t *seed_read, int32_t *seed_chain, int64_t seed_cap)
{
    const sa_src_t src = {sa, NULL};
    return mem_chain_src(opt, &src, l_pac, read_len, n_reads, mems, cap, n_mems, seeds, seed_read, seed_chain, seed_cap);
}
/* the same with SA lookups through an oracle FM-index (fmi_ref.c; full or lean form) */
int64_t oracle_mem_chain_fmi(const bsw_chain_opt_t *opt, const void *fmi, int64_t l_pac, const int32_t *read_len,
                             int32_t n_reads, const bsw_bwtintv_t *mems, int32_t cap, const int32_t *n_mems,
                             bsw_seed_t *seeds, int32_t *seed_read, int32_t *seed_chain, int64_t seed_cap)
{
    const sa_src_t src = {NULL, fmi};
    return mem_chain_src(opt, &src, l_pac, read_len, n_reads, mems, cap, n_mems, seeds, seed_read, seed_chain, seed_cap);
}
static int64_t mem_chain_src(const bsw_chain_opt_t *opt, const sa_src_t *sa, int64_t l_pac, const int32_t *read_len,
                             int32_t n_reads, const bsw_bwtintv_t *mems, int32_t cap, const int32_t *n_mems,
                             bsw_seed_t *seeds, int32_t *seed_read, int32_t *seed_chain, int64_t seed_cap)
{
    int64_t ns = 0;
    for (int32_t r = 0; r < n_reads; ++r) {
        ochain_t *a = NULL;
        const int nm = n_mems[r] < cap ? n_mems[r] : cap;
        int nc = read_chains(opt, sa, l_pac, read_len[r], mems + (size_t)r * cap, nm, &a);
        nc = chain_flt(opt, nc, a);
        for (int c = 0; c < nc; ++c) {
            for (int j = 0; j < a[c].n; ++j, ++ns) {
                if (ns < seed_cap) {
                    seeds[ns].rbeg = a[c].seeds[j].rbeg;
                    seeds[ns].qbeg = a[c].seeds[j].qbeg;
                    seeds[ns].len = a[c].seeds[j].len;
                    seed_read[ns] = r;
                    seed_chain[ns] = c;
                }
            }
            free(a[c].seeds);
        }
        free(a);
    }
    return ns;
}
