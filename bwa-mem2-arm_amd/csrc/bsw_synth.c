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
