/*
 * bsw_batch.h -- ".bswb" SeqPair batch files: record / replay of getScores16/8 batches
 * (SURVEY.md §8(f) row 3).
 *
 * A batch as upstream hands it to BandedPairWiseSW::getScores16/8 (SeqPair AoS + seqBufRef +
 * seqBufQer, docs-archive/WEEK1_WRAPPER_COMPLETE.md:259-269) plus the scoring and band it was
 * run with, optionally with the outputs an engine produced.  Purpose: capture real batches
 * from an upstream build elsewhere (the shim records them when BSW_RECORD is set) and replay
 * them here for parity and benchmarking without network access.
 *
 * Layout (little endian):
 *   bswb_header_t (128 bytes)
 *   SeqPair[n_pairs]            56 bytes each (include/bsw_seqpair.h)
 *   uint8_t ref[ref_bytes]      codes 0..4 (seqBufRef)
 *   uint8_t qer[qer_bytes]      codes 0..4 (seqBufQer)
 * checksum = FNV-1a 64 over everything after the header.
 */
#ifndef BSW_BATCH_H
#define BSW_BATCH_H

#include <stdint.h>
#include "bsw.h"

#ifdef __cplusplus
extern "C" {
#endif

#define BSWB_MAGIC   0x42575342u   /* "BSWB" */
#define BSWB_VERSION 1u
#define BSWB_HAS_OUTPUTS 1u        /* flags: SeqPair outputs (score .. max_off) are valid      */

typedef struct bswb_header_t {
    uint32_t magic, version;
    uint32_t header_bytes;         /* 128                                                      */
    uint32_t flags;
    int64_t  n_pairs, ref_bytes, qer_bytes;
    uint64_t checksum;
    int32_t  w, cell_bits;
    bsw_params_t params;           /* 6 x int32 + 25 + 3 x int8 = 52 bytes                      */
    uint8_t  reserved[128 - 48 - 8 - sizeof(bsw_params_t)];
} bswb_header_t;

/* Write a batch (has_outputs: the SeqPairs' output fields are meaningful).  0 or BSW_E*. */
int bswb_write(const char *path, const bsw_params_t *params, int32_t w, int32_t cell_bits,
               int has_outputs, const SeqPair *pairs, int64_t n_pairs, const uint8_t *ref,
               int64_t ref_bytes, const uint8_t *qer, int64_t qer_bytes);

/* Read the header (validates magic / version / sizes against the file length). */
int bswb_read_header(const char *path, bswb_header_t *h);

/* Read the payload into caller buffers sized from the header; verifies the checksum
 * (BSW_E_RANGE on mismatch). */
int bswb_read(const char *path, bswb_header_t *h, SeqPair *pairs, uint8_t *ref, uint8_t *qer);

#ifdef __cplusplus
}
#endif
#endif /* BSW_BATCH_H */
