/*
 * bsw_seqpair.h -- the SeqPair record of BWA-MEM2's seed-extension batch API.
 *
 * Byte-compatible with upstream bwa-mem2 v2.2.1 `src/bandedSWA.h` `struct dnaSeqPair`
 * (14 x int32 = 56 B), the struct the fork's `getScores16/getScores8` take
 * (reference: docs-archive/WEEK1_WRAPPER_COMPLETE.md:259-269; field list: SURVEY.md
 * Appendix B, upstream recall, no upstream header exists in /root/reference).
 *
 * If a translation unit already includes upstream's bandedSWA.h, define
 * BSW_HAVE_UPSTREAM_SEQPAIR before including this file so the two
 * definitions do not collide; the static asserts below pin the layout.
 */
#ifndef BSW_SEQPAIR_H
#define BSW_SEQPAIR_H

#include <stdint.h>
#include <stddef.h>

#ifndef BSW_HAVE_UPSTREAM_SEQPAIR
typedef struct dnaSeqPair {
    int32_t idr, idq, id;     /* offsets of ref / query in seqBufRef / seqBufQer; pair id    */
    int32_t len1, len2;       /* ref (target, DP rows) length, query (DP columns) length   */
    int32_t h0;               /* initial score: seed score (left ext) / left score (right)  */
    int32_t seqid, regid;     /* caller bookkeeping (read index, region index); untouched   */
    int32_t score, tle, gtle, qle;   /* outputs                                             */
    int32_t gscore, max_off;         /* outputs                                             */
} SeqPair;
#endif

#ifdef __cplusplus
static_assert(sizeof(SeqPair) == 56, "SeqPair must be 56 bytes (upstream layout)");
static_assert(offsetof(SeqPair, len1) == 12 && offsetof(SeqPair, h0) == 20, "SeqPair input layout");
static_assert(offsetof(SeqPair, score) == 32 && offsetof(SeqPair, max_off) == 52, "SeqPair output layout");
#else
_Static_assert(sizeof(SeqPair) == 56, "SeqPair must be 56 bytes (upstream layout)");
_Static_assert(offsetof(SeqPair, score) == 32 && offsetof(SeqPair, max_off) == 52, "SeqPair output layout");
#endif

/* Byte offsets used by device code and the ctypes mirror. */
#define BSW_SP_IDR 0
#define BSW_SP_IDQ 4
#define BSW_SP_LEN1 12
#define BSW_SP_LEN2 16
#define BSW_SP_H0 20
#define BSW_SP_SCORE 32
#define BSW_SP_WORDS 14

/* Upstream constants (bandedSWA.h). */
#define BSW_AMBIG 4            /* code of N; scores w_ambig (-1) against anything          */
#define BSW_MAX_SEQ_LEN8 128   /* upstream's 8-bit path length cap (HEAP_CORRUPTION_FIX.md:46) */

#endif /* BSW_SEQPAIR_H */
