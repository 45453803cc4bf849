/*
 * fmi_ref.c -- TEST INFRASTRUCTURE (CPU oracle), never linked into the product.
 *
 * Restatement of BWA-MEM's FM-index seeding ("FM-index SMEM seeding";
 * the reference's motivation: PHASE4_SEEDING_ANALYSIS.md:32-66 names bwt_smem1 / bwt_extend /
 * mem_collect_intv in src/FMI_search.cpp and src/bwamem.cpp as the seeding hot spots).  The
 * reference repository holds no source of these functions, so they are restated here from the
 * published upstream algorithms [UPSTREAM-RECALL]:
 *   - lh3/bwa bwt.c  bwt_smem1a(), bwt_seed_strategy1(), bwt_extend()/bwt_set_intv() -- the SMEM
 *     search that bwa-mem2 v2.2.1 (the fork's base) documents as output-identical;
 *   - lh3/bwa bwamem.c mem_collect_intv() -- the three seeding passes (SMEMs; re-seeding inside
 *     long, low-occurrence SMEMs with min_intv = s + 1; LAST-like seeds) and the final sort by
 *     info;
 *   - bwa-mem2 src/FMI_search.cpp conventions for the index: the BWT of T$ with T = ref +
 *     reverse-complement(ref) keeps the sentinel, count[c] = 1 + #{bases < c} (the +1 is '$'),
 *     occurrence counts over 64-base CP_OCC blocks, intervals [k, k + s) 0-based, and
 *     backwardExt()'s sentinel_offset rule for the reverse-complement interval l.
 *
 * Everything is written for clarity, not speed: the suffix array is a comparison sort of whole
 * suffixes (independent of the product's prefix-doubling builder), occurrences come from a
 * plain prefix-count table (independent of the product's one-hot blocks), and the SMEM passes
 * are literal transcriptions of the loops above (vectors of intervals, bwt_reverse_intvs, ...).
 * Parity of the restatement against the reference itself is UNPINNED (no upstream fixtures);
 * tests/test_fmi.py pins it against brute-force string search instead.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int64_t n;            /* |T| = 2 * ref_len; T$ has n + 1 suffixes                          */
    uint8_t *t;           /* T[0, n) codes 0..3  (NULL in the lean form)                        */
    int64_t *sa;          /* SA[0, n] (SA[0] = n, the '$' suffix)  (NULL in the lean form)      */
    uint8_t *bwt;         /* BWT[0, n]: T[SA[r] - 1] or 4 for '$'                               */
    int64_t *occ;         /* occ[4 * r + c] = #c in BWT[0, r), r in [0, n + 1]  (full form)     */
    int64_t count[5];     /* count[c] = 1 + #{T[i] < c}                                         */
    int64_t sentinel;     /* r with SA[r] == 0 (BWT[r] = '$')                                   */
    /* lean form (a genome-sized index in ~1.8 B per row instead of 42): occurrence checkpoints
     * every LEAN_CP rows (cp[4 * b + c] = #c in BWT[0, b * LEAN_CP)) + a scan of at most 63 BWT
     * bytes per query, and SA sampled every LEAN_SA rows resolved by LF walks (bwa's bwt_sa) */
    int lean;
    int64_t *cp;
    int64_t *ssa;
} fmi_ref_t;
#define LEAN_CP 64
#define LEAN_SA 32

typedef struct { uint64_t x[3]; uint64_t info; } ref_intv_t;   /* bwa's bwtintv_t */

static const uint8_t *g_t;
static int64_t g_n;

/* suffix comparison on T$ ('$' smaller than every base) */
static int cmp_suffix(const void *pa, const void *pb)
{
    int64_t a = *(const int64_t *)pa, b = *(const int64_t *)pb;
    while (a < g_n && b < g_n) {
        if (g_t[a] != g_t[b]) return g_t[a] < g_t[b] ? -1 : 1;
        ++a; ++b;
    }
    /* the shorter remainder reaches '$' first and is smaller */
    return (a == g_n) ? (b == g_n ? 0 : -1) : 1;
}

/* Build the index of ref[0, len) (codes 0..3; ambiguous bases must already be replaced, as
 * bwa's .pac does).  Returns 0, or -1 on a bad code / allocation failure. */
int oracle_fmi_build(const uint8_t *ref, int64_t len, fmi_ref_t *f)
{
    memset(f, 0, sizeof(*f));
    int64_t n = 2 * len;
    f->n = n;
    f->t = (uint8_t *)malloc(n > 0 ? n : 1);
    f->sa = (int64_t *)malloc(sizeof(int64_t) * (n + 1));
    f->bwt = (uint8_t *)malloc(n + 1);
    f->occ = (int64_t *)malloc(sizeof(int64_t) * 4 * (n + 2));
    if (!f->t || !f->sa || !f->bwt || !f->occ) return -1;
    for (int64_t i = 0; i < len; ++i) {
        if (ref[i] > 3) return -1;
        f->t[i] = ref[i];
        f->t[n - 1 - i] = (uint8_t)(3 - ref[i]);      /* reverse complement */
    }
    for (int64_t i = 0; i <= n; ++i) f->sa[i] = i;
    g_t = f->t; g_n = n;
    qsort(f->sa, (size_t)(n + 1), sizeof(int64_t), cmp_suffix);
    for (int64_t r = 0; r <= n; ++r) {
        f->bwt[r] = f->sa[r] == 0 ? 4 : f->t[f->sa[r] - 1];
        if (f->sa[r] == 0) f->sentinel = r;
    }
    for (int c = 0; c < 4; ++c) f->occ[c] = 0;
    for (int64_t r = 0; r <= n; ++r)
        for (int c = 0; c < 4; ++c) f->occ[4 * (r + 1) + c] = f->occ[4 * r + c] + (f->bwt[r] == c);
    int64_t tot[4] = {0, 0, 0, 0};
    for (int64_t i = 0; i < n; ++i) tot[f->t[i]]++;
    f->count[0] = 1;
    for (int c = 0; c < 4; ++c) f->count[c + 1] = f->count[c] + tot[c];
    return 0;
}

/* The same index from a caller-supplied suffix array of T$ (n + 1 entries): the bench's CPU
 * baseline leg uses the product's suffix array to skip the comparison sort on large
 * references; the tests build with oracle_fmi_build (and compare the two arrays). */
int oracle_fmi_build_with_sa(const uint8_t *ref, int64_t len, const int64_t *sa, fmi_ref_t *f)
{
    memset(f, 0, sizeof(*f));
    int64_t n = 2 * len;
    f->n = n;
    f->t = (uint8_t *)malloc(n > 0 ? n : 1);
    f->sa = (int64_t *)malloc(sizeof(int64_t) * (n + 1));
    f->bwt = (uint8_t *)malloc(n + 1);
    f->occ = (int64_t *)malloc(sizeof(int64_t) * 4 * (n + 2));
    if (!f->t || !f->sa || !f->bwt || !f->occ) return -1;
    for (int64_t i = 0; i < len; ++i) {
        if (ref[i] > 3) return -1;
        f->t[i] = ref[i];
        f->t[n - 1 - i] = (uint8_t)(3 - ref[i]);
    }
    memcpy(f->sa, sa, sizeof(int64_t) * (n + 1));
    for (int64_t r = 0; r <= n; ++r) {
        f->bwt[r] = f->sa[r] == 0 ? 4 : f->t[f->sa[r] - 1];
        if (f->sa[r] == 0) f->sentinel = r;
    }
    for (int c = 0; c < 4; ++c) f->occ[c] = 0;
    for (int64_t r = 0; r <= n; ++r)
        for (int c = 0; c < 4; ++c) f->occ[4 * (r + 1) + c] = f->occ[4 * r + c] + (f->bwt[r] == c);
    int64_t tot[4] = {0, 0, 0, 0};
    for (int64_t i = 0; i < n; ++i) tot[f->t[i]]++;
    f->count[0] = 1;
    for (int c = 0; c < 4; ++c) f->count[c + 1] = f->count[c] + tot[c];
    return 0;
}

void oracle_fmi_free(fmi_ref_t *f)
{
    free(f->t); free(f->sa); free(f->bwt); free(f->occ); free(f->cp); free(f->ssa);
    memset(f, 0, sizeof(*f));
}

static int64_t occ(const fmi_ref_t *f, int c, int64_t r)
{
    if (!f->lean) return f->occ[4 * r + c];
    const int64_t b = r / LEAN_CP;
    int64_t v = f->cp[4 * b + c];
    for (int64_t i = b * LEAN_CP; i < r; ++i) v += f->bwt[i] == c;
    return v;
}

/* The lean form from a caller-supplied suffix array of T$ (the bench's CPU leg at genome scale,
 * where the full form's 42 B per row would need ~250 GB): BWT codes, occurrence checkpoints and
 * the sampled SA are derived with `nthreads` threads; the SA array itself is not kept. */
#include <pthread.h>
typedef struct { fmi_ref_t *f; const uint8_t *ref; int64_t len; const int64_t *sa; int64_t r0, r1; int64_t cnt[4]; } lean_job_t;
static void *lean_worker(void *pa)
{
    lean_job_t *j = (lean_job_t *)pa;
    fmi_ref_t *f = j->f;
    const int64_t n = f->n;
    for (int64_t r = j->r0; r < j->r1; ++r) {
        const int64_t p = j->sa[r];
        uint8_t c = 4;
        if (p > 0) {
            const int64_t i = p - 1;                          /* T[i]: forward or reverse strand */
            c = i < j->len ? j->ref[i] : (uint8_t)(3 - j->ref[n - 1 - i]);
        }
        f->bwt[r] = c;
        if (r % LEAN_SA == 0) f->ssa[r / LEAN_SA] = p;
    }
    /* per-block counts of this range (blocks are whole: r0 is a multiple of LEAN_CP) */
    for (int64_t b = j->r0 / LEAN_CP; b * LEAN_CP < j->r1; ++b) {
        int64_t c4[4] = {0, 0, 0, 0};
        const int64_t e = (b + 1) * LEAN_CP < j->r1 ? (b + 1) * LEAN_CP : j->r1;
        for (int64_t r = b * LEAN_CP; r < e; ++r)
            if (f->bwt[r] < 4) c4[f->bwt[r]]++;
        for (int c = 0; c < 4; ++c) f->cp[4 * (b + 1) + c] = c4[c];   /* counts of block b, prefixed below */
    }
    return NULL;
}
int oracle_fmi_build_lean(const uint8_t *ref, int64_t len, const int64_t *sa, int nthreads, fmi_ref_t *f)
{
    memset(f, 0, sizeof(*f));
    const int64_t n = 2 * len, N = n + 1, nb = N / LEAN_CP + 1;
    f->n = n;
    f->lean = 1;
    f->bwt = (uint8_t *)malloc((size_t)N);
    f->cp = (int64_t *)calloc((size_t)(4 * (nb + 1)), sizeof(int64_t));
    f->ssa = (int64_t *)malloc(sizeof(int64_t) * (size_t)(N / LEAN_SA + 1));
    if (!f->bwt || !f->cp || !f->ssa) return -1;
    int64_t tot[4] = {0, 0, 0, 0};
    for (int64_t i = 0; i < len; ++i) {
        if (ref[i] > 3) return -1;
        tot[ref[i]]++;
        tot[3 - ref[i]]++;                                    /* the reverse complement's base */
    }
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    lean_job_t jobs[64];
    pthread_t th[64];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (lean_job_t){f, ref, len, sa, (N * t / nthreads) / LEAN_CP * LEAN_CP,
                               t + 1 == nthreads ? N : (N * (t + 1) / nthreads) / LEAN_CP * LEAN_CP, {0}};
        pthread_create(&th[t], NULL, lean_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    for (int64_t b = 1; b <= nb; ++b)                          /* block counts -> prefix counts */
        for (int c = 0; c < 4; ++c) f->cp[4 * b + c] += f->cp[4 * (b - 1) + c];
    for (int64_t r = 0; r < N; ++r)
        if (f->bwt[r] == 4) { f->sentinel = r; break; }
    f->count[0] = 1;
    for (int c = 0; c < 4; ++c) f->count[c + 1] = f->count[c] + tot[c];
    return 0;
}

/* SA[r]: the array (full form) or bwa's bwt_sa -- LF steps back to a sampled row (lean form) */
int64_t oracle_fmi_sa_at(const fmi_ref_t *f, int64_t r)
{
    if (!f->lean) return f->sa[r];
    int64_t steps = 0;
    while (r % LEAN_SA != 0) {
        const int c = f->bwt[r];
        if (c == 4) return steps;                             /* the '$' row: SA = 0 */
        r = f->count[c] + occ(f, c, r);
        ++steps;
    }
    return f->ssa[r / LEAN_SA] + steps;
}

/* 64-row occurrence blocks an extension touches (1 when rows k and k + s share one, else 2):
 * the algorithmic HBM bytes of the GPU kernel's block layout, counted for bench.py's roofline */
static uint64_t g_block_loads, g_ext_calls;
void oracle_fmi_counters(uint64_t *out, int reset)
{
    out[0] = __atomic_load_n(&g_ext_calls, __ATOMIC_RELAXED);
    out[1] = __atomic_load_n(&g_block_loads, __ATOMIC_RELAXED);
    if (reset) { g_ext_calls = 0; g_block_loads = 0; }
}
/* the same split by seeding phase (0 pass-1 forward, 1 pass-1 backward sweep, 2 / 3 pass-2
 * forward / backward, 4 pass 3): [phase][0] extensions, [1] those of an interval with s >= 2 (the
 * GPU kernel's text mode serves s = 1 from the text), [2] block loads of the s >= 2 ones */
static __thread int g_phase;
static uint64_t g_ph[5][3];
/* analysis counters (tools/smem_phase_counts.py), per phase, over the extensions the GPU kernel
 * walks through occurrence blocks -- s >= 2 and a result string longer than kt (shorter ones come
 * from its k-mer table): [0] all of them, [1] those of an interval with exactly s = 2, [2] those
 * of [1] that keep s = 2 (both occurrences agree on the next base: what a two-position text mode
 * would serve) */
static __thread int g_len;
static int g_kt;
static uint64_t g_s2[5][3];
void oracle_fmi_s2_counters(uint64_t *out15, int reset, int kt)
{
    for (int p = 0; p < 5; ++p)
        for (int k = 0; k < 3; ++k) {
            out15[3 * p + k] = __atomic_load_n(&g_s2[p][k], __ATOMIC_RELAXED);
            if (reset) g_s2[p][k] = 0;
        }
    g_kt = kt;
}
void oracle_fmi_phase_counters(uint64_t *out15, int reset)
{
    for (int p = 0; p < 5; ++p)
        for (int k = 0; k < 3; ++k) {
            out15[3 * p + k] = __atomic_load_n(&g_ph[p][k], __ATOMIC_RELAXED);
            if (reset) g_ph[p][k] = 0;
        }
}

/* bwa-mem2 FMI_search::backwardExt: interval (k, l, s) of string X -> that of aX */
static void backward_ext(const fmi_ref_t *f, const uint64_t in[3], int a, uint64_t out[3])
{
    int64_t k[4], l[4], s[4];
    int64_t sp = (int64_t)in[0], ep = (int64_t)in[0] + (int64_t)in[2];
    __atomic_fetch_add(&g_ext_calls, 1, __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_block_loads, (sp >> 6) == (ep >> 6) ? 1 : 2, __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_ph[g_phase][0], 1, __ATOMIC_RELAXED);
    if (in[2] >= 2) {
        __atomic_fetch_add(&g_ph[g_phase][1], 1, __ATOMIC_RELAXED);
        __atomic_fetch_add(&g_ph[g_phase][2], (sp >> 6) == (ep >> 6) ? 1 : 2, __ATOMIC_RELAXED);
    }
    for (int b = 0; b < 4; ++b) {
        k[b] = f->count[b] + occ(f, b, sp);
        s[b] = occ(f, b, ep) - occ(f, b, sp);
    }
    int64_t sentinel_offset = (sp <= f->sentinel && ep > f->sentinel) ? 1 : 0;
    l[3] = (int64_t)in[1] + sentinel_offset;
    l[2] = l[3] + s[3];
    l[1] = l[2] + s[2];
    l[0] = l[1] + s[1];
    if (in[2] >= 2 && g_len > g_kt) {
        __atomic_fetch_add(&g_s2[g_phase][0], 1, __ATOMIC_RELAXED);
        if (in[2] == 2) __atomic_fetch_add(&g_s2[g_phase][1], 1, __ATOMIC_RELAXED);
        if (in[2] == 2 && s[a] == 2) __atomic_fetch_add(&g_s2[g_phase][2], 1, __ATOMIC_RELAXED);
    }
    out[0] = (uint64_t)k[a]; out[1] = (uint64_t)l[a]; out[2] = (uint64_t)s[a];
}

/* bwt_extend(is_back = 1) restricted to base c, and is_back = 0 (forward by base c = the
 * complement of the read base: backward extension of the reverse-complement interval) */
static void ext_back(const fmi_ref_t *f, const ref_intv_t *ik, int c, ref_intv_t *ok)
{
    backward_ext(f, ik->x, c, ok->x);
}
static void ext_fwd(const fmi_ref_t *f, const ref_intv_t *ik, int c, ref_intv_t *ok)
{
    uint64_t sw[3] = {ik->x[1], ik->x[0], ik->x[2]}, o[3];
    backward_ext(f, sw, c, o);
    ok->x[0] = o[1]; ok->x[1] = o[0]; ok->x[2] = o[2];
}

static void set_intv(const fmi_ref_t *f, int c, ref_intv_t *ik)
{
    ik->x[0] = (uint64_t)f->count[c];
    ik->x[2] = (uint64_t)(f->count[c + 1] - f->count[c]);
    ik->x[1] = (uint64_t)f->count[3 - c];
    ik->info = 0;
}

typedef struct { int64_t n, m; ref_intv_t *a; } ivec_t;
static void ipush(ivec_t *v, const ref_intv_t *x)
{
    if (v->n == v->m) {
        v->m = v->m ? 2 * v->m : 16;
        v->a = (ref_intv_t *)realloc(v->a, sizeof(ref_intv_t) * v->m);
    }
    v->a[v->n++] = *x;
}
static void ireverse(ivec_t *v)
{
    for (int64_t i = 0; i < v->n / 2; ++i) {
        ref_intv_t t = v->a[i]; v->a[i] = v->a[v->n - 1 - i]; v->a[v->n - 1 - i] = t;
    }
}

/* bwt_smem1a: SMEMs of q[0, len) overlapping position x (min_intv, max_intv as upstream);
 * returns the start of the next search (end of the longest forward match). */
static int smem1a(const fmi_ref_t *f, int len, const uint8_t *q, int x, int min_intv, uint64_t max_intv,
                  ivec_t *mem, ivec_t *prev, ivec_t *curr)
{
    int i, j, c, ret;
    ref_intv_t ik, ok;
    ivec_t *swap;
    mem->n = 0;
    if (q[x] > 3) return x + 1;
    if (min_intv < 1) min_intv = 1;
    set_intv(f, q[x], &ik);
    ik.info = (uint64_t)(x + 1);
    for (i = x + 1, curr->n = 0; i < len; ++i) {            /* forward search */
        if (ik.x[2] < max_intv) {
            ipush(curr, &ik);
            break;
        } else if (q[i] < 4) {
            c = 3 - q[i];
            g_len = i + 1 - x;
            ext_fwd(f, &ik, c, &ok);
            if (ok.x[2] != ik.x[2]) {
                ipush(curr, &ik);
                if (ok.x[2] < (uint64_t)min_intv) break;
            }
            ik = ok; ik.info = (uint64_t)(i + 1);
        } else {
            ipush(curr, &ik);
            break;
        }
    }
    if (i == len) ipush(curr, &ik);
    g_phase |= 1;
    ireverse(curr);
    ret = (int)(uint32_t)curr->a[0].info;
    swap = curr; curr = prev; prev = swap;
    for (i = x - 1; i >= -1; --i) {                           /* backward search for MEMs */
        c = i < 0 ? -1 : q[i] < 4 ? q[i] : -1;
        for (j = 0, curr->n = 0; j < prev->n; ++j) {
            ref_intv_t *p = &prev->a[j];
            g_len = (int)(uint32_t)p->info - i;
            if (c >= 0 && ik.x[2] >= max_intv) ext_back(f, p, c, &ok);
            if (c < 0 || ik.x[2] < max_intv || ok.x[2] < (uint64_t)min_intv) {
                if (curr->n == 0) {
                    if (mem->n == 0 || (uint64_t)(i + 1) < (mem->a[mem->n - 1].info >> 32)) {
                        ik = *p; ik.info |= (uint64_t)(i + 1) << 32;
                        ipush(mem, &ik);
                    }
                }
            } else if (curr->n == 0 || ok.x[2] != curr->a[curr->n - 1].x[2]) {
                ok.info = p->info;
                ipush(curr, &ok);
            }
        }
        if (curr->n == 0) break;
        swap = curr; curr = prev; prev = swap;
    }
    ireverse(mem);
    g_phase &= ~1;
    return ret;
}

/* bwt_seed_strategy1: the LAST-like pass */
static int seed_strategy1(const fmi_ref_t *f, int len, const uint8_t *q, int x, int min_len, int max_intv,
                          ref_intv_t *mem)
{
    int i, c;
    ref_intv_t ik, ok;
    memset(mem, 0, sizeof(*mem));
    if (q[x] > 3) return x + 1;
    set_intv(f, q[x], &ik);
    for (i = x + 1; i < len; ++i) {
        if (q[i] < 4) {
            c = 3 - q[i];
            g_len = i + 1 - x;
            ext_fwd(f, &ik, c, &ok);
            if (ok.x[2] < (uint64_t)max_intv && i - x >= min_len) {
                *mem = ok;
                mem->info = (uint64_t)x << 32 | (uint64_t)(i + 1);
                return i + 1;
            }
            ik = ok;
        } else {
            return i + 1;
        }
    }
    return len;
}

typedef struct {
    int32_t min_seed_len, split_width, max_mem_intv;
    float split_factor;
} oracle_mem_opt_t;

/* deterministic final order: info, then k, s, l (upstream's introsort leaves ties unordered) */
static int cmp_intv(const void *pa, const void *pb)
{
    const ref_intv_t *a = (const ref_intv_t *)pa, *b = (const ref_intv_t *)pb;
    if (a->info != b->info) return a->info < b->info ? -1 : 1;
    if (a->x[0] != b->x[0]) return a->x[0] < b->x[0] ? -1 : 1;
    if (a->x[2] != b->x[2]) return a->x[2] < b->x[2] ? -1 : 1;
    if (a->x[1] != b->x[1]) return a->x[1] < b->x[1] ? -1 : 1;
    return 0;
}

/* mem_collect_intv for one read: writes up to cap intervals into out, returns how many there
 * are (> cap: truncated). */
int oracle_collect_intv(const fmi_ref_t *f, const oracle_mem_opt_t *opt, const uint8_t *seq, int len,
                        ref_intv_t *out, int cap)
{
    int i, k, x = 0, old_n;
    int split_len = (int)(opt->min_seed_len * opt->split_factor + .499);
    ivec_t mem = {0, 0, 0}, mem1 = {0, 0, 0}, t0 = {0, 0, 0}, t1 = {0, 0, 0};
    g_phase = 0;
    while (x < len) {                                         /* first pass: SMEMs */
        if (seq[x] < 4) {
            x = smem1a(f, len, seq, x, 1, 0, &mem1, &t0, &t1);
            for (i = 0; i < mem1.n; ++i) {
                ref_intv_t *p = &mem1.a[i];
                int slen = (int)((uint32_t)p->info - (p->info >> 32));
                if (slen >= opt->min_seed_len) ipush(&mem, p);
            }
        } else {
            ++x;
        }
    }
    old_n = (int)mem.n;                                       /* second pass: re-seeding */
    g_phase = 2;
    for (k = 0; k < old_n; ++k) {
        ref_intv_t p = mem.a[k];
        int start = (int)(p.info >> 32), end = (int)(uint32_t)p.info;
        if (end - start < split_len || p.x[2] > (uint64_t)opt->split_width) continue;
        smem1a(f, len, seq, (start + end) >> 1, (int)p.x[2] + 1, 0, &mem1, &t0, &t1);
        for (i = 0; i < mem1.n; ++i)
            if ((int)((uint32_t)mem1.a[i].info - (mem1.a[i].info >> 32)) >= opt->min_seed_len)
                ipush(&mem, &mem1.a[i]);
    }
    g_phase = 4;
    if (opt->max_mem_intv > 0) {                              /* third pass: LAST-like */
        x = 0;
        while (x < len) {
            if (seq[x] < 4) {
                ref_intv_t m;
                x = seed_strategy1(f, len, seq, x, opt->min_seed_len, opt->max_mem_intv, &m);
                if (m.x[2] > 0) ipush(&mem, &m);
            } else {
                ++x;
            }
        }
    }
    if (mem.n) qsort(mem.a, (size_t)mem.n, sizeof(ref_intv_t), cmp_intv);   /* qsort(NULL, 0): UB */
    int n = (int)mem.n;
    for (i = 0; i < n && i < cap; ++i) out[i] = mem.a[i];
    free(mem.a); free(mem1.a); free(t0.a); free(t1.a);
    return n;
}

/* many reads (read i = reads[off[i], off[i] + len[i])), cap intervals per read at out + i * cap;
 * cnt[i] = interval count of read i */
void oracle_collect_intv_batch(const fmi_ref_t *f, const oracle_mem_opt_t *opt, const uint8_t *reads,
                               const int64_t *off, const int32_t *len, int32_t n, ref_intv_t *out,
                               int32_t cap, int32_t *cnt)
{
    for (int32_t i = 0; i < n; ++i)
        cnt[i] = oracle_collect_intv(f, opt, reads + off[i], len[i], out + (int64_t)i * cap, cap);
}

/* the same over nthreads pthreads (CPU baseline leg of bench.py): reads split round-robin in
 * blocks of 256 */
#include <pthread.h>
typedef struct {
    const fmi_ref_t *f; const oracle_mem_opt_t *opt; const uint8_t *reads; const int64_t *off;
    const int32_t *len; int32_t n; ref_intv_t *out; int32_t cap; int32_t *cnt; int tid, nt;
} cib_arg_t;
static void *cib_worker(void *pa)
{
    cib_arg_t *a = (cib_arg_t *)pa;
    for (int32_t b = a->tid * 256; b < a->n; b += a->nt * 256)
        for (int32_t i = b; i < b + 256 && i < a->n; ++i)
            a->cnt[i] = oracle_collect_intv(a->f, a->opt, a->reads + a->off[i], a->len[i],
                                            a->out + (int64_t)i * a->cap, a->cap);
    return 0;
}
void oracle_collect_intv_mt(const fmi_ref_t *f, const oracle_mem_opt_t *opt, const uint8_t *reads,
                            const int64_t *off, const int32_t *len, int32_t n, ref_intv_t *out,
                            int32_t cap, int32_t *cnt, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    cib_arg_t *args = (cib_arg_t *)malloc(sizeof(cib_arg_t) * nthreads);
    for (int t = 0; t < nthreads; ++t) {
        cib_arg_t a = {f, opt, reads, off, len, n, out, cap, cnt, t, nthreads};
        args[t] = a;
        pthread_create(&th[t], 0, cib_worker, &args[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], 0);
    free(th); free(args);
}

/* accessors for the Python binding */
int64_t oracle_fmi_n(const fmi_ref_t *f) { return f->n; }
int64_t oracle_fmi_sentinel(const fmi_ref_t *f) { return f->sentinel; }
void oracle_fmi_count(const fmi_ref_t *f, int64_t *c5) { memcpy(c5, f->count, sizeof(f->count)); }
void oracle_fmi_sa(const fmi_ref_t *f, int64_t *sa)
{
    if (!f->lean) { memcpy(sa, f->sa, sizeof(int64_t) * (f->n + 1)); return; }
    for (int64_t r = 0; r <= f->n; ++r) sa[r] = oracle_fmi_sa_at(f, r);
}
void oracle_fmi_sa_rows(const fmi_ref_t *f, const int64_t *rows, int64_t m, int64_t *out)
{
    for (int64_t i = 0; i < m; ++i) out[i] = oracle_fmi_sa_at(f, rows[i]);
}
void oracle_fmi_bwt(const fmi_ref_t *f, uint8_t *bwt) { memcpy(bwt, f->bwt, (size_t)f->n + 1); }
size_t oracle_fmi_sizeof(void) { return sizeof(fmi_ref_t); }
