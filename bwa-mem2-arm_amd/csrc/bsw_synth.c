/*
 * bsw_synth.c -- deterministic synthetic SeqPair batches (bench + tests tooling).
 *
 * Workload of BASELINE.json configs[1] / SURVEY.md §8(d): each pair is a 300 bp uniform
 * ACGT reference window with 0.1% N, and a query that is the window's first 150 bp with
 * 2% substitutions and 0.2% 1-3 bp indels; 10% of pairs get an unrelated random query
 * (early z-drop / m==0 termination).  h0 uniform in [h0_lo, h0_hi].  RNG: splitmix64,
 * seed 42 by default (echoing benchmark_threading.sh:45,59's random.seed(42)); every
 * pair draws from its own stream (seed, pair index), so batches are reproducible
 * and can be generated in parallel or in shards (pair_base).
 *
 * Layout is upstream's: SeqPair AoS + two concatenated 1-byte-per-base code buffers
 * (codes 0..3 = ACGT, 4 = N); idr = i*tlen, idq = i*qlen.
 */
#include <stdint.h>
#include <string.h>
#include "../../include/bsw_seqpair.h"

static inline uint64_t splitmix64(uint64_t *s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
/* uniform in [0,1) with 53 bits */
static inline double u01(uint64_t *s) { return (double)(splitmix64(s) >> 11) * (1.0 / 9007199254740992.0); }
static inline uint32_t below(uint64_t *s, uint32_t n) { return (uint32_t)(((splitmix64(s) >> 32) * (uint64_t)n) >> 32); }

typedef struct bsw_synth_cfg {
    uint64_t seed;
    int32_t tlen, qlen;         /* ref window / query lengths (300 / 150 at C2)          */
    int32_t h0_lo, h0_hi;       /* inclusive                                              */
    double p_sub, p_indel;      /* per-base substitution / indel-start probability        */
    double p_unrelated;         /* fraction of pairs with an unrelated random query       */
    double p_n;                 /* per-base N rate in the reference                        */
} bsw_synth_cfg;

void bsw_synth_default(bsw_synth_cfg *c)
{
    c->seed = 42;
    c->tlen = 300;
    c->qlen = 150;
    c->h0_lo = 19;
    c->h0_hi = 100;
    c->p_sub = 0.02;
    c->p_indel = 0.002;
    c->p_unrelated = 0.10;
    c->p_n = 0.001;
}

/* Generate pairs [pair_base, pair_base + n) into pairs[0..n), ref[0..n*tlen),
 * qer[0..n*qlen).  Offsets (idr/idq) are local to these buffers; id = global index. */
void bsw_synth_batch(const bsw_synth_cfg *c, int64_t pair_base, int32_t n, SeqPair *pairs,
                     uint8_t *ref, uint8_t *qer)
{
    const int32_t T = c->tlen, Q = c->qlen;
    for (int32_t k = 0; k < n; ++k) {
        int64_t gi = pair_base + k;
        uint64_t s = c->seed * 0x2545F4914F6CDD1Dull ^ ((uint64_t)gi * 0x9E3779B97F4A7C15ull);
        splitmix64(&s);
        uint8_t *r = ref + (int64_t)k * T;
        uint8_t *q = qer + (int64_t)k * Q;
        for (int32_t i = 0; i < T; ++i) r[i] = (u01(&s) < c->p_n) ? 4 : (uint8_t)below(&s, 4);
        if (u01(&s) < c->p_unrelated) {
            for (int32_t j = 0; j < Q; ++j) q[j] = (uint8_t)below(&s, 4);
        } else {
            int32_t i = 0, j = 0;
            while (j < Q) {
                double u = u01(&s);
                if (u < c->p_indel) {
                    int32_t l = 1 + (int32_t)below(&s, 3);
                    if (splitmix64(&s) & 1) { /* insertion in the query */
                        for (int32_t t = 0; t < l && j < Q; ++t) q[j++] = (uint8_t)below(&s, 4);
                    } else {                   /* deletion from the query */
                        i += l;
                    }
                    continue;
                }
                uint8_t b = (i < T) ? r[i] : (uint8_t)below(&s, 4);
                ++i;
                if (u < c->p_indel + c->p_sub && b < 4) b = (uint8_t)((b + 1 + below(&s, 3)) & 3);
                q[j++] = b;
            }
        }
        SeqPair *p = &pairs[k];
        memset(p, 0, sizeof(*p));
        p->idr = (int32_t)((int64_t)k * T);
        p->idq = (int32_t)((int64_t)k * Q);
        p->id = (int32_t)gi;
        p->len1 = T;
        p->len2 = Q;
        p->h0 = c->h0_lo + (int32_t)below(&s, (uint32_t)(c->h0_hi - c->h0_lo + 1));
        p->seqid = (int32_t)gi;
        p->regid = 0;
    }
}

/* ------------------------------------------------------------------ read-level workload
 * C4/C5-shaped input for the extension pipeline (include/bsw_ext.h): a random reference and
 * reads sampled from it with an edit script, each with ONE exact-match seed, as upstream's
 * SMEM seeding would hand to mem_chain2aln.  Reads are forward-strand (the extension math is
 * strand-independent).  A fraction p_unrelated of reads are random sequence with a planted
 * 19..30 bp exact copy of a random reference position: a spurious seed hit whose extensions
 * die early (the mis-seeded case the z-drop handles). */
typedef struct bsw_seed_s { int64_t rbeg; int32_t qbeg; int32_t len; } bsw_seed_s; /* = bsw_seed_t */

void bsw_synth_reference(uint64_t seed, int64_t len, double p_n, uint8_t *out)
{
    /* 64K-base blocks, each from its own stream: reproducible and parallelisable */
    const int64_t B = 65536;
    for (int64_t b0 = 0; b0 < len; b0 += B) {
        uint64_t s = seed * 0x2545F4914F6CDD1Dull ^ ((uint64_t)(b0 / B + 1) * 0xD1B54A32D192ED03ull);
        splitmix64(&s);
        const int64_t e = b0 + B < len ? b0 + B : len;
        for (int64_t i = b0; i < e; ++i) out[i] = (u01(&s) < p_n) ? 4 : (uint8_t)below(&s, 4);
    }
}

typedef struct bsw_reads_cfg {
    uint64_t seed;
    int32_t read_len;           /* 150                                                   */
    int32_t min_seed;           /* 19 (bwa -k)                                           */
    double p_sub, p_indel;      /* per-base substitution / indel-start probability       */
    double p_unrelated;         /* reads with a spurious planted seed                    */
} bsw_reads_cfg;

void bsw_reads_default(bsw_reads_cfg *c)
{
    c->seed = 42;
    c->read_len = 150;
    c->min_seed = 19;
    c->p_sub = 0.02;
    c->p_indel = 0.002;
    c->p_unrelated = 0.10;
}

/* Reads [read_base, read_base + n): reads[k*read_len ..], seeds[k], origin[k] (may be NULL).
 * Returns the number of reads that got a seed (seeds[k].len == 0 otherwise). */
int32_t bsw_synth_reads(const bsw_reads_cfg *c, const uint8_t *ref, int64_t ref_len, int64_t read_base,
                        int32_t n, uint8_t *reads, bsw_seed_s *seeds, int64_t *origin)
{
    const int32_t L = c->read_len;
    int32_t nseeded = 0;
    int64_t rp[4096];
    if (L > 4096 || ref_len < 2 * (int64_t)L + 64) return -1;
    for (int32_t k = 0; k < n; ++k) {
        const int64_t gi = read_base + k;
        uint64_t s = c->seed * 0x9E3779B97F4A7C15ull ^ ((uint64_t)gi * 0xBF58476D1CE4E5B9ull) ^ 0x5555;
        splitmix64(&s);
        uint8_t *q = reads + (int64_t)k * L;
        bsw_seed_s *sd = &seeds[k];
        sd->rbeg = 0; sd->qbeg = 0; sd->len = 0;
        const int64_t org = (int64_t)(u01(&s) * (double)(ref_len - L - 64));
        if (origin) origin[k] = org;
        if (u01(&s) < c->p_unrelated) {
            for (int32_t j = 0; j < L; ++j) q[j] = (uint8_t)below(&s, 4);
            const int32_t sl = 19 + (int32_t)below(&s, 12);
            const int32_t qb = (int32_t)below(&s, (uint32_t)(L - sl + 1));
            int64_t rb = (int64_t)(u01(&s) * (double)(ref_len - sl));
            int ok = 1;
            for (int32_t t = 0; t < sl; ++t) { q[qb + t] = ref[rb + t]; if (ref[rb + t] > 3) ok = 0; }
            if (ok) { sd->rbeg = rb; sd->qbeg = qb; sd->len = sl; ++nseeded; }
            continue;
        }
        /* edit script: rp[j] = reference position read base j copies (-1: inserted) */
        int64_t i = org;
        int32_t j = 0;
        while (j < L) {
            const double u = u01(&s);
            if (u < c->p_indel) {
                const int32_t l = 1 + (int32_t)below(&s, 3);
                if (splitmix64(&s) & 1) {
                    for (int32_t t = 0; t < l && j < L; ++t) { rp[j] = -1; q[j++] = (uint8_t)below(&s, 4); }
                } else {
                    i += l;
                }
                continue;
            }
            uint8_t b = ref[i];
            if (u01(&s) < c->p_sub) b = (uint8_t)((b < 4 ? b : 0) + 1 + below(&s, 3)) & 3;
            rp[j] = i;
            q[j++] = b;
            ++i;
        }
        /* longest run of consecutive reference positions with identical, non-N bases */
        int32_t best = 0, bq = 0, run = 0;
        for (int32_t t = 0; t < L; ++t) {
            const int ok = rp[t] >= 0 && ref[rp[t]] < 4 && q[t] == ref[rp[t]];
            if (!ok) run = 0;
            else if (run > 0 && rp[t] == rp[t - 1] + 1) ++run;
            else run = 1;
            if (run > best) { best = run; bq = t - run + 1; }
        }
        if (best >= c->min_seed) {
            sd->rbeg = rp[bq]; sd->qbeg = bq; sd->len = best; ++nseeded;
        }
    }
    return nseeded;
}

/* Paired-end reads with SEVERAL seeds per read (C4/C5, closer to what upstream's SMEM
 * seeding + chaining hand to mem_chain2aln_across_reads_V2).  Read pair k covers fragment
 * [p, p + I) of the reference, I uniform in [ins_lo, ins_hi]: read 2k = the fragment's first
 * read_len bases, read 2k+1 its last read_len bases in forward-strand orientation (the
 * reverse-complemented mate as the extension sees it; the extension math is strand-free).
 * Each read gets its own substitution / indel script.  Seeds: EVERY maximal exact run of
 * >= min_seed bases along the read's true alignment path (one chain of up to 8 seeds, longest
 * first, as chaining orders them); with probability p_spurious an extra 19..30 bp exact copy
 * of a random reference position is planted in the read (a second, spurious chain); a
 * fraction p_unrelated of reads are random sequence with only such a planted seed.
 * Output: reads[r * read_len ..] for r in [0, 2 n_pairs), seeds[0..ns) with seed_read[k] =
 * the read (relative to this call) of seed k, grouped by read, and seed_chain[k] = 0 for the
 * read's true chain, 1 for a planted spurious seed on a true read (chains in bwa's order: the
 * heavier one first); returns ns (<= 9 per read), -1 if the reference is too short. */
int32_t bsw_synth_pe_seeds(const bsw_reads_cfg *c, const uint8_t *ref, int64_t ref_len, int64_t pair_base,
                           int32_t n_pairs, int32_t ins_lo, int32_t ins_hi, double p_spurious,
                           uint8_t *reads, bsw_seed_s *seeds, int32_t *seed_read, int32_t *seed_chain)
{
    const int32_t L = c->read_len;
    int64_t rp[4096];
    int32_t ns = 0;
    if (L > 4096 || ins_hi < L || ref_len < (int64_t)ins_hi + 2 * (int64_t)L + 64) return -1;
    for (int32_t k = 0; k < n_pairs; ++k) {
        const int64_t gi = pair_base + k;
        uint64_t s = c->seed * 0x9E3779B97F4A7C15ull ^ ((uint64_t)gi * 0x94D049BB133111EBull) ^ 0xA5A5;
        splitmix64(&s);
        const int32_t ins = ins_lo + (int32_t)below(&s, (uint32_t)(ins_hi - ins_lo + 1));
        const int64_t frag = (int64_t)(u01(&s) * (double)(ref_len - ins - 64));
        for (int m = 0; m < 2; ++m) {
            const int32_t rid = 2 * k + m;
            uint8_t *q = reads + (int64_t)rid * L;
            const int64_t org = m == 0 ? frag : frag + ins - L;
            int32_t first = ns;
            if (u01(&s) < c->p_unrelated) {          /* random read, one planted spurious seed */
                for (int32_t j = 0; j < L; ++j) q[j] = (uint8_t)below(&s, 4);
            } else {
                int64_t i = org;
                int32_t j = 0;
                while (j < L) {
                    const double u = u01(&s);
                    if (u < c->p_indel) {
                        const int32_t l = 1 + (int32_t)below(&s, 3);
                        if (splitmix64(&s) & 1) {
                            for (int32_t t = 0; t < l && j < L; ++t) { rp[j] = -1; q[j++] = (uint8_t)below(&s, 4); }
                        } else {
                            i += l;
                        }
                        continue;
                    }
                    uint8_t b = ref[i];
                    if (u01(&s) < c->p_sub) b = (uint8_t)((b < 4 ? b : 0) + 1 + below(&s, 3)) & 3;
                    rp[j] = i;
                    q[j++] = b;
                    ++i;
                }
                /* maximal runs of consecutive matching reference positions (non-N) */
                int32_t run = 0;
                for (int32_t t = 0; t <= L; ++t) {
                    const int ok = t < L && rp[t] >= 0 && ref[rp[t]] < 4 && q[t] == ref[rp[t]] &&
                                   (run == 0 || rp[t] == rp[t - 1] + 1);
                    if (ok) { ++run; continue; }
                    if (run >= c->min_seed && ns - first < 8) {
                        seeds[ns].qbeg = t - run; seeds[ns].rbeg = rp[t - run]; seeds[ns].len = run;
                        seed_chain[ns] = 0;
                        seed_read[ns++] = rid;
                    }
                    run = (t < L && rp[t] >= 0 && ref[rp[t]] < 4 && q[t] == ref[rp[t]]) ? 1 : 0;
                }
                /* longest first (chaining's order) */
                for (int32_t a = first + 1; a < ns; ++a)
                    for (int32_t b2 = a; b2 > first && seeds[b2].len > seeds[b2 - 1].len; --b2) {
                        bsw_seed_s t2 = seeds[b2]; seeds[b2] = seeds[b2 - 1]; seeds[b2 - 1] = t2;
                        /* seed_read / seed_chain are equal within the run */
                    }
                if (!(u01(&s) < p_spurious)) continue;
            }
            /* planted spurious seed: exact copy of a random reference position */
            const int32_t sl = 19 + (int32_t)below(&s, 12);
            const int32_t qb = (int32_t)below(&s, (uint32_t)(L - sl + 1));
            const int64_t rb = (int64_t)(u01(&s) * (double)(ref_len - sl));
            int ok = 1;
            for (int32_t t = 0; t < sl; ++t) { q[qb + t] = ref[rb + t]; if (ref[rb + t] > 3) ok = 0; }
            /* true seeds overlapping the planted bases are no longer exact: drop them */
            int32_t w2 = first;
            for (int32_t a = first; a < ns; ++a)
                if (seeds[a].qbeg + seeds[a].len <= qb || seeds[a].qbeg >= qb + sl) {
                    seeds[w2] = seeds[a]; seed_chain[w2] = seed_chain[a]; seed_read[w2++] = seed_read[a];
                }
            ns = w2;
            if (ok) {
                seeds[ns].rbeg = rb; seeds[ns].qbeg = qb; seeds[ns].len = sl;
                seed_chain[ns] = ns > first ? 1 : 0;
                seed_read[ns++] = rid;
            }
        }
    }
    return ns;
}

/* ---------------------------------------------------------------- mate-rescue jobs
 * Jobs shaped like mem_matesw's (bwamem_pair.cpp; include/bsw_mate.h): the mate read
 * (read_len bases sampled from the reference with substitutions / short indels) against a
 * reference window of win_len bases -- insert-size window [mean - 4 sd, mean + 4 sd] plus
 * the read length -- that holds the mate's true origin with probability p_true (a random
 * window otherwise: the mate is unmapped or elsewhere).  pairs[k]: idr = window start in
 * ref (seqBufRef = the reference), idq = k * read_len in qer, len1 = win_len,
 * len2 = read_len, h0 = xtra = KSW_XSUBO | KSW_XSTART | (read_len * a < 250 ? KSW_XBYTE : 0)
 * | min_seed * a, exactly bwa's mate-rescue flags for match score a. */
typedef struct bsw_mates_cfg {
    uint64_t seed;
    int32_t read_len, win_len;   /* 150, 550                                             */
    int32_t a, min_seed;         /* match score 1, bwa -k 19                             */
    double p_true;               /* window holds the mate (0.8)                          */
    double p_sub, p_indel;       /* read edit rates (0.02, 0.002)                        */
} bsw_mates_cfg;

void bsw_mates_default(bsw_mates_cfg *c)
{
    c->seed = 42;
    c->read_len = 150;
    c->win_len = 550;
    c->a = 1;
    c->min_seed = 19;
    c->p_true = 0.8;
    c->p_sub = 0.02;
    c->p_indel = 0.002;
}

int32_t bsw_synth_mates(const bsw_mates_cfg *c, const uint8_t *ref, int64_t ref_len, int64_t base, int32_t n,
                        SeqPair *pairs, uint8_t *qer)
{
    const int32_t L = c->read_len, W = c->win_len;
    if (L <= 0 || W < L || ref_len < (int64_t)W + 2 * L + 64) return -1;
    const int32_t xtra = 0x40000 | 0x80000 | (L * c->a < 250 ? 0x10000 : 0) | ((c->min_seed * c->a) & 0xffff);
    int32_t ntrue = 0;
    for (int32_t k = 0; k < n; ++k) {
        const int64_t gi = base + k;
        uint64_t s = c->seed * 0xA0761D6478BD642Full ^ ((uint64_t)gi * 0xE7037ED1A0B428DBull) ^ 0x3333;
        splitmix64(&s);
        const int64_t org = (int64_t)(u01(&s) * (double)(ref_len - W - L - 64)) + L;
        uint8_t *q = qer + (int64_t)k * L;
        int64_t i = org;
        int32_t j = 0;
        while (j < L) {
            if (u01(&s) < c->p_indel) {
                const int32_t l = 1 + (int32_t)below(&s, 3);
                if (splitmix64(&s) & 1) {
                    for (int32_t t = 0; t < l && j < L; ++t) q[j++] = (uint8_t)below(&s, 4);
                } else {
                    i += l;
                }
                continue;
            }
            uint8_t b = ref[i++];
            if (u01(&s) < c->p_sub) b = (uint8_t)((b < 4 ? b : 0) + 1 + below(&s, 3)) & 3;
            q[j++] = b;
        }
        int64_t w0;
        if (u01(&s) < c->p_true) {
            w0 = org - (int64_t)below(&s, (uint32_t)(W - L + 1));
            if (w0 < 0) w0 = 0;
            ++ntrue;
        } else {
            w0 = (int64_t)(u01(&s) * (double)(ref_len - W));
        }
        SeqPair *p = &pairs[k];
        memset(p, 0, sizeof(*p));
        p->idr = (int32_t)w0;
        p->idq = (int32_t)((int64_t)k * L);
        p->id = (int32_t)gi;
        p->len1 = W;
        p->len2 = L;
        p->h0 = xtra;
    }
    return ntrue;
}

/* ---------------------------------------------------------------- global (CIGAR) jobs
 * Jobs shaped like bwa_gen_cigar2's ksw_global2 calls (mem_reg2aln, src/bwa.cpp;
 * include/bsw_global.h): a read of read_len bases sampled from the reference with
 * substitutions / short indels, against exactly the reference span it covers (rb..re), band w
 * by bwa_gen_cigar2's rule with opt->w = w_cap.  pairs[k]: idr = span start in ref (seqBufRef =
 * the reference), idq = k * read_len in qer, len1 = span length, len2 = read_len, h0 = w. */
typedef struct bsw_globals_cfg {
    uint64_t seed;
    int32_t read_len, w_cap;     /* 150, opt->w = 100                                    */
    int32_t a, o_del, e_del, o_ins, e_ins;   /* bwa defaults 1, 6, 1, 6, 1               */
    double p_sub, p_indel;       /* read edit rates (0.02, 0.002)                        */
} bsw_globals_cfg;

void bsw_globals_default(bsw_globals_cfg *c)
{
    c->seed = 42;
    c->read_len = 150;
    c->w_cap = 100;
    c->a = 1;
    c->o_del = c->o_ins = 6;
    c->e_del = c->e_ins = 1;
    c->p_sub = 0.02;
    c->p_indel = 0.002;
}

static int32_t gen_cigar_band(int l_query, int rlen, int w_, int a, int o_del, int e_del, int o_ins, int e_ins)
{
    int max_ins = (int)((double)(((l_query + 1) >> 1) * a - o_ins) / e_ins + 1.);
    int max_del = (int)((double)(((l_query + 1) >> 1) * a - o_del) / e_del + 1.);
    int max_gap = max_ins > max_del ? max_ins : max_del;
    int d = rlen > l_query ? rlen - l_query : l_query - rlen;
    max_gap = max_gap > 1 ? max_gap : 1;
    int w = (max_gap + d + 1) >> 1;
    w = w < w_ ? w : w_;
    return w > d + 3 ? w : d + 3;
}

int32_t bsw_synth_globals(const bsw_globals_cfg *c, const uint8_t *ref, int64_t ref_len, int64_t base, int32_t n,
                          SeqPair *pairs, uint8_t *qer)
{
    const int32_t L = c->read_len;
    if (L <= 0 || ref_len < 4 * (int64_t)L + 64) return -1;
    for (int32_t k = 0; k < n; ++k) {
        const int64_t gi = base + k;
        uint64_t s = c->seed * 0x8EBC6AF09C88C6E3ull ^ ((uint64_t)gi * 0x589965CC75374CC3ull) ^ 0x5555;
        splitmix64(&s);
        const int64_t org = (int64_t)(u01(&s) * (double)(ref_len - 3 * L - 64));
        uint8_t *q = qer + (int64_t)k * L;
        int64_t i = org;
        int32_t j = 0;
        while (j < L) {
            if (j > 0 && j < L - 4 && u01(&s) < c->p_indel) {       /* no indel at the read ends */
                const int32_t l = 1 + (int32_t)below(&s, 3);
                if (splitmix64(&s) & 1) {
                    for (int32_t t = 0; t < l && j < L - 1; ++t) q[j++] = (uint8_t)below(&s, 4);
                } else {
                    i += l;
                }
                continue;
            }
            uint8_t b = ref[i++];
            if (u01(&s) < c->p_sub) b = (uint8_t)((b < 4 ? b : 0) + 1 + below(&s, 3)) & 3;
            q[j++] = b;
        }
        SeqPair *p = &pairs[k];
        memset(p, 0, sizeof(*p));
        p->idr = (int32_t)org;
        p->idq = (int32_t)((int64_t)k * L);
        p->id = (int32_t)gi;
        p->len1 = (int32_t)(i - org);
        p->len2 = L;
        p->h0 = gen_cigar_band(L, p->len1, c->w_cap, c->a, c->o_del, c->e_del, c->o_ins, c->e_ins);
    }
    return 0;
}
