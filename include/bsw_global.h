/*
 * bsw_global.h -- batched banded GLOBAL alignment with traceback:
 * upstream ksw_global2 semantics on MI355X, one call per batch.
 *
 * Replaces, per batch of final alignments (mem_reg2aln -> bwa_gen_cigar2, src/bwa.cpp):
 *   int ksw_global2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
 *                   const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
 *                   int *n_cigar, uint32_t **cigar)        -- src/ksw.cpp [UPSTREAM-RECALL,
 *   SURVEY.md §2 row 3], called once per alignment with w from bsw_gen_cigar_band() below.
 * bwa-mem2 keeps this call scalar and per alignment; here a whole batch of alignments (all
 * regions of a chunk of reads) goes to the GPU in one call.
 *
 * Job i = pairs[i]: query = seqBufQer[idq, idq + len2), target = seqBufRef[idr, idr + len1),
 * band w = pairs[i].h0 (>= 0).  Results:
 *   pairs[i].score       = ksw_global2's return value (other SeqPair outputs untouched)
 *   cigar[i * cigar_stride + k], k < n_cigar[i]: the CIGAR exactly as ksw_global2 returns it
 *                          (len << 4 | op; op 0 = M, 1 = I, 2 = D)
 *   n_cigar[i]           = op count; -1 if more than cigar_stride ops (score still valid);
 *                          -2 if len2 >= 1, len1 >= 1 and len2 < len1 - w: there the upstream
 *                          traceback starts outside the band and reads outside the row's
 *                          backtrack columns (no defined result; bwa_gen_cigar2's w >= |len1 -
 *                          len2| + 3 never asks for it)
 * cigar == NULL (cigar_stride 0): scores only, no traceback matrix.
 * Scoring = the context's bsw_params_t (mat, o_del, e_del, o_ins, e_ins; zdrop / end_bonus
 * unused).  Codes 0..4 (4 = N).  Limits: len1, len2 <= BSW_MAX_LEN.
 */
#ifndef BSW_GLOBAL_H
#define BSW_GLOBAL_H

#include <stdint.h>
#include <stdlib.h>
#include "bsw.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Blocking host-buffer call on the context's first device. */
int bsw_ksw_global2(bsw_ctx_t *ctx, SeqPair *pairs, const uint8_t *seqBufRef, const uint8_t *seqBufQer,
                    int32_t n, uint32_t *cigar, int32_t cigar_stride, int32_t *n_cigar);

/* Device-resident form: every pointer in HBM of the context's first device, `stream` a
 * hipStream_t or NULL.  Returns when scores, CIGARs and counts are in HBM. */
int bsw_ksw_global2_device(bsw_ctx_t *ctx, SeqPair *d_pairs, const uint8_t *d_ref, const uint8_t *d_qer,
                           int32_t n, uint32_t *d_cigar, int32_t cigar_stride, int32_t *d_n_cigar,
                           void *stream);

typedef struct bsw_global_stats_t {
    float   kernel_ms;          /* DP + traceback kernels (HIP events, same stream)            */
    int32_t n_jobs;             /* jobs in the call                                            */
    int32_t n_lane, n_wide;     /* jobs on the register kernel / the int32 HBM-row kernel       */
    int32_t n_launches;
    int64_t cells;              /* band cells computed (sum over jobs of row band widths)      */
    int64_t z_bytes;            /* traceback-matrix bytes written (nibble per cell, per wave)   */
    int32_t n_tb_retry;         /* column-kernel jobs whose traceback left the narrow corridor
                                   window (or whose corridor does not fit it) and were rerun with
                                   the full band window (ABI version 7)                        */
    int32_t pad_;
} bsw_global_stats_t;
int bsw_global_last_stats(bsw_ctx_t *ctx, bsw_global_stats_t *out);

/* bwa_gen_cigar2's band width (src/bwa.cpp) for a query of l_query bases against a reference
 * span of rlen bases, with opt->w = w_ and match score a = mat[0]. */
static inline int bsw_gen_cigar_band(int l_query, int rlen, int w_, int a, int o_del, int e_del,
                                     int o_ins, int e_ins)
{
    int max_ins = (int)((double)(((l_query + 1) >> 1) * a - o_ins) / e_ins + 1.);
    int max_del = (int)((double)(((l_query + 1) >> 1) * a - o_del) / e_del + 1.);
    int max_gap = max_ins > max_del ? max_ins : max_del;
    int w, min_w;
    max_gap = max_gap > 1 ? max_gap : 1;
    w = (max_gap + abs(rlen - l_query) + 1) >> 1;
    w = w < w_ ? w : w_;
    min_w = abs(rlen - l_query) + 3;
    return w > min_w ? w : min_w;
}

#ifdef __cplusplus
}
#endif
#endif /* BSW_GLOBAL_H */
