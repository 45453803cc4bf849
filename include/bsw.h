/*
 * bsw.h -- C ABI of the MI355X-native seed-extension engine (banded Smith-Waterman,
 * BWA-MEM2 `BandedPairWiseSW::getScores16/getScores8` semantics = `ksw_extend2`).
 *
 * Plain pointers and sizes only (no torch, no HIP types in the signatures), so an
 * upstream bwa-mem2 build, a ctypes loader or any FFI can bind it.  Every entry point
 * below names the reference interface it replaces:
 *
 *   bsw_create        <- BandedPairWiseSW::BandedPairWiseSW(o_del, e_del, o_ins, e_ins,
 *                        zdrop, end_bonus, mat, w_match, w_mismatch, numThreads)
 *                        (call site: docs-archive/INTEGRATION_COMPLETE.md:61-63)
 *   bsw_destroy       <- BandedPairWiseSW::~BandedPairWiseSW (frees the F8_/H8_ scratch,
 *                        PHASE2_WEEK1_WEEK2_COMPLETE.md:83-98)
 *   bsw_get_scores    <- getScores16 / getScores8 (SeqPair*, uint8_t *seqBufRef,
 *                        uint8_t *seqBufQer, int32_t numPairs, uint16_t numThreads,
 *                        int32_t w)   (docs-archive/WEEK1_WRAPPER_COMPLETE.md:259-269)
 *                        with cell_bits = 16 or 8 selecting the entry point.
 *   bsw_get_scores_device   device-resident form of the same call (inputs already in
 *                        HBM; what bench.py times).  No upstream counterpart.
 *
 * Semantics: for every pair p in [0, n) the outputs p.score, p.tle, p.gtle, p.qle,
 * p.gscore, p.max_off are bit-identical to scalar `ksw_extend2(qlen=len2,
 * query=seqBufQer+idq, tlen=len1, target=seqBufRef+idr, m=5, mat, o_del, e_del, o_ins,
 * e_ins, w, end_bonus, zdrop, h0, ...)`.  Inputs are base codes 0..4 (4 = N).
 * Unlike upstream, nothing is written to pairs[n .. roundUp(n, SIMD_WIDTH)).
 *
 * Errors: every call returns 0 or a negative BSW_E* code; nothing throws; nothing
 * falls back to the CPU (there is no CPU path in the product).  The C++ shim
 * (bandedSWA_gpu.h) keeps upstream's `void` + fprintf/exit convention on top.
 * Thread safety: bsw_get_scores may be called concurrently on one context (upstream
 * calls getScores* from kt_for workers); each call takes its own stream + buffers.
 */
#ifndef BSW_H
#define BSW_H

#include <stdint.h>
#include "bsw_seqpair.h"

#ifdef __cplusplus
extern "C" {
#endif

#define BSW_ABI_VERSION 8

enum {
    BSW_OK = 0,
    BSW_E_INVAL = -22,      /* bad argument (null pointer, n < 0, bad cell_bits, bad params) */
    BSW_E_NOMEM = -12,      /* device or pinned host allocation failed                      */
    BSW_E_NODEV = -19,      /* no HIP device / device index out of range                    */
    BSW_E_HIP = -5,         /* a HIP runtime call or kernel launch failed                   */
    BSW_E_RANGE = -34       /* a pair exceeds a supported size (len > BSW_MAX_LEN)          */
};

#define BSW_MAX_LEN 32767     /* per-sequence length limit (int16 cell range, upstream MAX_SEQ_LEN16) */

/* Scoring parameters: the upstream BandedPairWiseSW constructor arguments. */
typedef struct bsw_params_t {
    int32_t o_del, e_del, o_ins, e_ins;   /* gap open / extend (positive penalties)   */
    int32_t zdrop;                        /* z-drop; <= 0 disables                      */
    int32_t end_bonus;                    /* opt->pen_clip5 at the call site            */
    int8_t  mat[25];                      /* 5x5 score matrix [target*5 + query]       */
    int8_t  w_match, w_mismatch;          /* opt->a, -opt->b (kept for the shim)       */
    int8_t  w_ambig;                      /* score vs N; upstream DEFAULT_AMBIG = -1   */
} bsw_params_t;

typedef struct bsw_ctx bsw_ctx_t;

/* Fill *p with bwa-mem defaults: -A1 -B4 -O6,6 -E1,1 -d100 -L5 (mat = bwa_fill_scmat). */
void bsw_params_default(bsw_params_t *p);

/* Create an engine on HIP devices [device0, device0 + n_gpus).  n_gpus >= 1.
 * Multi-device policy of host-buffer calls: a call of fewer than BSW_OPT_SPLIT_MIN pairs
 * (default 131072) runs whole on one device -- the one with the fewest calls in flight, ties
 * rotating -- so concurrent kt_for-sized calls spread over the devices; larger calls are
 * split into contiguous pair ranges of equal static band cells, one per device. */
int  bsw_create(const bsw_params_t *params, int device0, int n_gpus, bsw_ctx_t **out);
/* The same over an explicit list: logical device k runs on HIP device devices[k].  Entries may
 * repeat (several logical devices with their own streams and buffers on one GPU): the
 * rehearsal form of an n-GPU context on a smaller box (ABI version 5). */
int  bsw_create_on(const bsw_params_t *params, const int *devices, int n_devices, bsw_ctx_t **out);
void bsw_destroy(bsw_ctx_t *ctx);

/* Blocking host-buffer call (drop-in for getScores16 / getScores8).
 * cell_bits: 16 -> int16 cells; 8 -> uint8 cells for pairs whose scores provably fit
 * (h0 + max(mat) * min(len1, len2) <= 255), int16 for the rest (overflow fallback).
 * Recovery (ABI version 7): when a device run fails with BSW_E_NOMEM or BSW_E_HIP the call is
 * run again before any error is returned -- once on the same device after its cached slots
 * (streams + buffers) are freed, then on each other device of the context, then -- for
 * BSW_E_NOMEM only (ABI 8: halving cannot cure a HIP error) -- in halves (recursively, down to
 * 4096 pairs), each half the same way.  Outputs are identical (pairs are
 * independent; a failed run writes no input field).  bsw_last_stats().recovery says which step
 * completed the call.  Upstream's plan for engine errors is to degrade, not abort
 * (PHASE2_IMPLEMENTATION_SUMMARY.md:210-225); there is still no CPU path. */
int  bsw_get_scores(bsw_ctx_t *ctx, SeqPair *pairs, const uint8_t *seqBufRef,
                    const uint8_t *seqBufQer, int32_t n, int32_t w, int cell_bits);

/* Device-resident call on the context's first device: d_pairs, d_ref and d_qer are
 * device pointers (idr / idq index d_ref / d_qer); results are written into d_pairs.
 * Runs on `stream` (a hipStream_t, or NULL for a stream of the context's own) and
 * returns when the results are in d_pairs (blocking, like getScores*). */
int  bsw_get_scores_device(bsw_ctx_t *ctx, SeqPair *d_pairs, const uint8_t *d_ref,
                           const uint8_t *d_qer, int32_t n, int32_t w, int cell_bits,
                           void *stream);

/* 2-bit wire form of a SeqPair batch (ABI version 7): the host pipeline's staging format made a
 * transport format, ~133 bytes per C2 pair instead of 56 + 450 -- what a batch scatter moves
 * between GPUs (bench.py's RCCL legs).  One buffer, offsets 256-aligned:
 *   [rec: n x 20 B {idr, idq, len1, len2, h0} | ref: 2-bit codes of the batch's ref extent + 4 pad
 *    | qer: the same for its qer extent | exc: one uint32 pos << 2 | (code & 15) >> 2 per byte
 *    outside 0..3 -- the code's low two bits are in the 2-bit plane (ref ones first, then qer
 *    ones, ascending; ABI 8, 28-bit positions with the whole nibble before)]
 * idr / idq are rebased to the extents (empty sequences: 0).  Extents must stay below 2^30 bytes
 * (exception positions are 30 bits): larger batches are packed in pieces. */
typedef struct bsw_packed_t {
    int32_t n;                            /* pairs                                        */
    int32_t n_exc_ref, n_exc_qer;         /* exception words of each extent               */
    int32_t pad_;
    int64_t ref_bytes, qer_bytes;         /* extent lengths (unpacked bytes)              */
    int64_t rec_off, ref_off, qer_off, exc_off, total_bytes;
} bsw_packed_t;
/* Host-only.  Fills *desc for pairs[0, n) over seqBufRef / seqBufQer; with dst == NULL only sizes
 * it (desc->total_bytes), else writes the packed batch into dst (cap bytes, >= total_bytes).
 * BSW_E_RANGE: a bad pair (negative or > BSW_MAX_LEN length, negative offset) or an extent past
 * 2^30 bytes. */
int  bsw_pack_batch(const SeqPair *pairs, const uint8_t *seqBufRef, const uint8_t *seqBufQer, int32_t n,
                    void *dst, int64_t cap, bsw_packed_t *desc);
/* Device-resident scoring of a packed batch on the context's first device: d_packed is the
 * buffer bsw_pack_batch wrote (desc its descriptor), now in HBM; the six outputs of pair p are
 * written to d_out[6p .. 6p+5] (score, tle, gtle, qle, gscore, max_off: 24 B per pair, the
 * gather's payload).  Unpack (one kernel), plan / sort / DP as bsw_get_scores_device, outputs
 * compacted.  Runs on `stream` (NULL: the context's own) and returns when d_out is written. */
int  bsw_get_scores_packed_device(bsw_ctx_t *ctx, const void *d_packed, const bsw_packed_t *desc,
                                  int32_t w, int cell_bits, int32_t *d_out, void *stream);

/* Per-call statistics of the last bsw_get_scores_device / bsw_get_scores on this
 * thread: the hot kernel's event-timed duration (ms) and the pairs routed per kernel. */
typedef struct bsw_stats_t {
    float   kernel_ms;          /* sum of DP-kernel durations (HIP events, same stream) */
    int32_t n_i16, n_u8, n_wide; /* pairs per kernel class                               */
    int32_t n_launches;         /* DP-kernel launches                                    */
    int32_t n_packed;           /* of n_i16 + n_u8: pairs run on the 8-bit-regime packed
                                   kernels (v_pk_* cells; ABI version 2)                 */
    float   stage_ms;           /* host-buffer calls: host time staging chunks into pinned
                                   memory (ABI version 4; 0 for device calls)            */
    float   host_ms;            /* host-buffer calls: wall time of the call on the device's
                                   host thread (staging + H2D + kernels + D2H)           */
    int32_t n_wave;             /* of n_i16: pairs run on the wave-per-alignment kernel
                                   (queries past 160 columns; ABI version 4)             */
    int32_t n_devices;          /* host-buffer calls: logical devices the call ran on
                                   (1, or all of them when split; ABI version 5)         */
    int32_t n_group;            /* of n_i16: pairs run on the small-batch row-group kernel
                                   (16 lanes per pair; ABI version 6)                    */
    int32_t recovery;           /* host-buffer calls: how a call whose first run failed with
                                   BSW_E_NOMEM / BSW_E_HIP was completed (ABI version 7):
                                   0 = no failure, 1 = rerun on its device after the cached
                                   slots were freed, 2 = rerun on another device of the
                                   context, 3 = rerun in halves (see bsw_get_scores)      */
} bsw_stats_t;
int  bsw_last_stats(bsw_ctx_t *ctx, bsw_stats_t *out);

/* Engine options: tuning and test knobs of one context (no upstream counterpart; upstream
 * has no such switches, so the defaults are the only production setting).  Set them before
 * the context is used by concurrent callers.  Returns BSW_E_INVAL for an unknown option or
 * an out-of-range value. */
enum {
    BSW_OPT_KERNEL8 = 1,      /* 8-bit-regime pairs (h0 + min(len1,len2) <= 255, bwa scoring):
                                 1 = packed-column kernel (default), 0 = int16 lane kernel,
                                 2 = packed-column kernel with byte-wide H/E planes (8-bit
                                 cells, fewer registers, more waves per SIMD; outputs are
                                 identical either way)                                         */
    BSW_OPT_FORK = 2,         /* a batch's class launches: 1 = fork over side streams
                                 (default), 0 = serial on the call's stream                   */
    BSW_OPT_SORTKEY = 3,      /* plan sort key: 1 = seed identities before h0 (default),
                                 0 = h0 only (scheduling only; results never change)          */
    BSW_OPT_GLOB_BAND = 4,    /* bsw_ksw_global2: 0 = column kernel first (default),
                                 1 = band kernel for every band-eligible job                  */
    BSW_OPT_EXT_CHUNK = 5,    /* extension calls: reads per chunk (0 = the int32-offset bound) */
    BSW_OPT_LONG = 7,         /* queries past the 160-column register kernels: 1 = one wavefront
                                 per alignment (bsw_wv.hip, default), 0 = the int32 wide kernel,
                                 2 = every pair the wave kernel can run goes there (tests)   */
    BSW_OPT_HOST_CHUNK = 6,   /* bsw_get_scores: largest pipeline chunk in pairs (default
                                 196608, rounded down to whole 4096-pair blocks, at least one):
                                 a host-buffer call is staged, copied and computed chunk by
                                 chunk over up to four slots so copies overlap the DP
                                 kernels; calls of <= 128K pairs run as one chunk            */
    BSW_OPT_HOST_PACK = 8,    /* bsw_get_scores staging of contiguous sequence buffers: 2 = 2-bit
                                 codes + exception words for bytes outside 0..3, 20-B input
                                 records, 24-B outputs back (default); 4 = nibbles + whole
                                 records (also the automatic fallback for chunks with > 1/32
                                 non-ACGT bytes); outputs are identical                      */
    BSW_OPT_SMALL_BATCH = 9,  /* calls (device calls, or host-buffer pipeline chunks) of at most
                                 this many pairs run every pair the wave-per-alignment kernel
                                 can take there (default 32768; 0 = off): a lane-per-pair wave
                                 lives ~1.2 ms at any batch size, a wave per alignment spreads
                                 the pair over 64 lanes -- kt_for-sized calls are latency-bound.
                                 Outputs are identical either way                              */
    BSW_OPT_SPLIT_MIN = 10,   /* contexts over several devices: host-buffer calls of fewer pairs
                                 (mate / global calls: jobs) run whole on one device (default
                                 131072; 0 = always split)                                    */
    BSW_OPT_COALESCE = 11,    /* host-buffer calls of at most this many pairs (default 8192; 0 =
                                 off) coalesce with concurrent callers on their device: queued
                                 calls of equal (w, cell_bits, end_bonus) run as ONE batch (one
                                 staging buffer, one plan / sort / DP, outputs scattered back);
                                 a lone caller runs at once.  (32768 until round 4: 8 callers x
                                 10K pairs measured 36-41 M/s coalesced vs a steady 40 direct;
                                 at 1K-4K coalescing is worth 1.5x.)  Outputs are identical
                                 either way                                                     */
    BSW_OPT_COALESCE_LEADERS = 12, /* coalesced batches in flight per device (1..16, default 4) */
    BSW_OPT_GROUP_KERNEL = 13, /* small batches (BSW_OPT_SMALL_BATCH): 1 = the row-group kernel
                                 (16 lanes per pair, queries <= 160, no plan / sort; default),
                                 0 = the planned path with the wave-per-alignment kernel.
                                 Outputs are identical either way                              */
    BSW_OPT_MID_BATCH = 14,   /* calls / chunks of more than BSW_OPT_SMALL_BATCH and at most this many
                                 pairs (default 32768; 0 = off) run on the row-group kernel's quad
                                 form (4 lanes per pair, targets <= 512 bytes) when
                                 BSW_OPT_GROUP_KERNEL is on -- an empty range at the defaults (the
                                 16-lane form measured faster up to 32K pairs; lower
                                 BSW_OPT_SMALL_BATCH to use it).  Outputs are identical either way */
    BSW_OPT_COALESCE_LINGER = 16, /* microseconds (0..100000, default 20): with more concurrent
                                 callers than BSW_OPT_COALESCE_LEADERS and two or more batches
                                 running, a new leader waits up to this long for 4096 queued pairs
                                 (or for fewer than two running batches) before taking the queue,
                                 so batches fill up.  Measured at 20 (round 6): 8 callers +15-30%
                                 at 1K-4K pairs per call, 16 callers equal or better (at 150,
                                 round 4: 4 / 16 callers mixed).  0 = off.  A lone
                                 caller never waits.  Outputs are identical                      */
    /* 15 and 17 (a busy-device routing knob and the persistent tile-queue kernel, ABI 7) were
       removed in ABI 8 after measuring slower than the defaults: BSW_E_INVAL */
    BSW_OPT_GQ32_MAX = 18,    /* batches of at most this many pairs (within BSW_OPT_SMALL_BATCH) run on
                                 the row-group kernel's 32-lane latency form (two DPP rows per pair);
                                 larger small batches on its 16-lane form.  Default 2048 (the
                                 crossover measured with 8 callers); 0 = off.
                                 Outputs are identical either way (ABI version 8)                */
    BSW_OPT_TEST_MISROUTE = 100, /* tests only: 1 = every pair to the QMAX=32 lane class, so
                                 any longer query trips the kernels' range guard (BSW_E_RANGE) */
    BSW_OPT_TEST_FAIL_ALLOC = 101 /* tests only: the next `value` (0..1000000) device buffer
                                 growths of the engine fail with hipErrorOutOfMemory, so the
                                 recovery of bsw_get_scores can be exercised.  The count is
                                 PROCESS-WIDE and consumed by every path's buffer growth (host-
                                 buffer and device calls, global / CIGAR, extension) of every
                                 context: set it only while one call runs                      */
};
int  bsw_set_option(bsw_ctx_t *ctx, int option, int64_t value);

/* Work-balanced split of one batch into `parts` contiguous pair ranges (what an n_gpus
 * context does inside bsw_get_scores, and what a one-process-per-GPU caller uses to shard a
 * batch across ranks): part k = pairs [cut[k], cut[k+1]), cut[0] = 0, cut[parts] = n, each
 * holding ~1/parts of the static band cells.  cut has parts + 1 entries.
 * Host-only arithmetic; needs no device. */
int  bsw_split_by_cells(const SeqPair *pairs, int32_t n, int32_t w, int32_t parts, int32_t *cut);

const char *bsw_strerror(int code);
int  bsw_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* BSW_H */
