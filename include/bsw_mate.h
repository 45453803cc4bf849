/*
 * bsw_mate.h -- batched local Smith-Waterman for mate rescue:
 * upstream ksw_align2 / ksw_u8 / ksw_i16 semantics on MI355X, one call per batch.
 *
 * Replaces, per batch of mate-rescue jobs built by mem_sam_pe_batch (src/bwamem_pair.cpp):
 *   kswv::getScores8 / getScores16 (SeqPair*, uint8_t *seqBufRef, uint8_t *seqBufQer,
 *       kswr_t *aln, int32_t numPairs, uint16_t numThreads, int32_t phase)
 *       -- docs-archive/INTEGRATION_COMPLETE.md:49-112, docs-archive/ARM-BATCHED-SAM-PLAN.md:34,
 *          8-bit / 16-bit split by KSW_XBYTE: docs-archive/WEEK1_BENCHMARK_RESULTS.md:97-103
 *   and the scalar fallback the fork uses for every 8-bit job
 *   ksw_align2(qlen, query, tlen, target, 5, mat, o_del, e_del, o_ins, e_ins, xtra, 0)
 *       -- docs-archive/WEEK2_STATUS.md:80-90, docs-archive/AWS_VALIDATION_SUCCESS.md:100-117.
 *
 * Job i = pairs[i]: target = seqBufRef[idr, idr + len1) (DP rows), query = seqBufQer[idq,
 * idq + len2) (DP columns), xtra = h0 (KSW_X* flags | 16-bit threshold, as ksw_align2 takes
 * it; bwa's mate rescue passes KSW_XSUBO | KSW_XSTART | (l_ms*a < 250 ? KSW_XBYTE : 0) |
 * min_seed_len*a).  aln[i] receives exactly ksw_align2's kswr_t: the forward pass
 * (score, te, qe, score2 / te2 of the best hit outside te +- score/max(mat) rows) and, with
 * KSW_XSTART, tb / qb from the reverse pass over the reversed prefixes.  KSW_XBYTE selects
 * ksw_u8 (16-lane striping, score capped at 255) over ksw_i16 (8 lanes); the two differ only
 * in those respects.  Codes 0..4 (4 = N).  Scoring = the context's bsw_params_t (mat, o_del,
 * e_del, o_ins, e_ins; zdrop / end_bonus unused).
 *
 * Limits: len2 <= BSW_MATE_MAX_QLEN (256), len1 <= BSW_MAX_LEN; o_ins >= 1 and max(mat) >= 1
 * (BSW_E_INVAL otherwise: with o_ins == 0 upstream's lazy-F early exit drops F chains in a
 * lane-order-dependent way the batch kernel does not reproduce).
 */
#ifndef BSW_MATE_H
#define BSW_MATE_H

#include <stdint.h>
#include "bsw.h"

#ifdef __cplusplus
extern "C" {
#endif

#define BSW_KSW_XBYTE  0x10000
#define BSW_KSW_XSTOP  0x20000
#define BSW_KSW_XSUBO  0x40000
#define BSW_KSW_XSTART 0x80000

#define BSW_MATE_MAX_QLEN 256

typedef struct bsw_kswr_t {          /* = upstream kswr_t                                     */
    int32_t score, te, qe;           /* best local score, its end on target / query (-1: none) */
    int32_t score2, te2;             /* best secondary hit (KSW_XSUBO) or -1                   */
    int32_t tb, qb;                  /* start (KSW_XSTART) or -1                               */
} bsw_kswr_t;

/* Blocking host-buffer call on the context's first device. */
int bsw_ksw_align2(bsw_ctx_t *ctx, const SeqPair *pairs, const uint8_t *seqBufRef,
                   const uint8_t *seqBufQer, int32_t n, bsw_kswr_t *aln);

/* Device-resident form: d_pairs / d_ref / d_qer / d_aln in HBM of the context's first device,
 * `stream` a hipStream_t or NULL.  Returns when d_aln holds the results. */
int bsw_ksw_align2_device(bsw_ctx_t *ctx, const SeqPair *d_pairs, const uint8_t *d_ref,
                          const uint8_t *d_qer, int32_t n, bsw_kswr_t *d_aln, void *stream);

typedef struct bsw_mate_stats_t {
    float   fwd_ms, rev_ms;          /* DP kernel time of the forward / reverse (XSTART) passes */
    int32_t n_fwd, n_rev;            /* jobs per pass                                          */
    int64_t cells_fwd;               /* DP cells of the forward pass (ncol * rows run)          */
} bsw_mate_stats_t;
int bsw_mate_last_stats(bsw_ctx_t *ctx, bsw_mate_stats_t *out);

#ifdef __cplusplus
}
#endif
#endif /* BSW_MATE_H */
