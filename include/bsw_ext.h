/*
 * bsw_ext.h -- seed-extension job builder + result interpreter on top of the batch engine
 * (upstream consumer row a9).
 *
 * Replaces the extension half of upstream bwa-mem2's per-chain alignment step
 * (mem_chain2aln / mem_chain2aln_across_reads_V2 in src/bwamem.cpp, the caller of
 * BandedPairWiseSW::getScores16/8 -- docs-archive/INTEGRATION_COMPLETE.md:16-63,
 * BUG_REPORT.md:28-41 for the call site), restated from bwa's ksw_extend2 consumer
 * [UPSTREAM-RECALL, SURVEY.md a9]:
 *
 *   seed (qbeg, rbeg, len) of a read of length l_query, seed score sc = len * a
 *   target window rmax = [min over the CHAIN's seeds of rbeg - qbeg - gap(qbeg),
 *                         max over the chain's seeds of rbeg + len + (l_query - qe) + gap(l_query - qe))
 *     clipped to [0, ref_len), gap(l) = min(max((l*a - o)/e + 1, 1), 2w)   (cal_max_gap); with
 *     opt->l_pac > 0 a window crossing l_pac keeps the side of the chain's first seed
 *     (mem_chain2aln's rmax[] computation).  bsw_extend_seeds treats every seed as a chain of one.
 *     Windows are clipped only at the strand boundary: the reference is ONE sequence (upstream
 *     also clips to the seed's contig, bns_fetch_seq; a multi-contig genome passed concatenated
 *     is extended across its contig joins -- see include/bsw_fmi.h "Scope").
 *   LEFT  (qbeg > 0): query = reverse(read[0, qbeg)), target = reverse(ref[rmax0, rbeg)),
 *         h0 = sc, end_bonus = pen_clip5, band w << k for k < max_band_try (retry while the
 *         score changed and max_off >= 3/4 of the band)
 *         local  if gscore <= 0 || gscore <= score - pen_clip5: qb = qbeg - qle, rb = rbeg - tle
 *         to-end otherwise:                                     qb = 0,          rb = rbeg - gtle
 *   RIGHT (qe = qbeg + len < l_query): query = read[qe, l_query), target = ref[rbeg + len, rmax1),
 *         h0 = the LEFT score (sc0), end_bonus = pen_clip3, same band retry
 *         local  if gscore <= 0 || gscore <= score - pen_clip3: qe += qle, re = rbeg + len + tle
 *         to-end otherwise:                                     qe = l_query, re = ... + gtle
 *   truesc accumulates the chosen (local or to-end) scores; w = widest band used.
 *
 * All LEFT extensions of a call form one batch (then one retry batch), then all RIGHT
 * extensions (their h0 depends on LEFT's result) -- the across-reads batching of
 * mem_chain2aln_across_reads_V2.  bsw_extend_seeds takes one seed per job (jobs of the same
 * read repeat its read_off / read_len); bsw_chain2aln below adds upstream's per-read chain /
 * seed order and contained-seed skipping on top.
 */
#ifndef BSW_EXT_H
#define BSW_EXT_H

#include <stdint.h>
#include "bsw.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bsw_seed_t {          /* one exact-match seed of read i (len == 0: no seed)     */
    int64_t rbeg;                    /* reference position of the seed's first base            */
    int32_t qbeg;                    /* read position of the seed's first base                 */
    int32_t len;
} bsw_seed_t;

typedef struct bsw_ext_opt_t {
    int32_t w;                       /* band width (bwa -w, default 100)                        */
    int32_t pen_clip5, pen_clip3;    /* clipping penalties (bwa -L, default 5,5)                */
    int32_t max_band_try;            /* band doublings incl. the first try (bwa: 2)             */
    int64_t l_pac;                   /* > 0: ref is bwa's forward + reverse-complement text of
                                        2 * l_pac bases (bns->l_pac), and a target window that
                                        crosses l_pac keeps the strand of the chain's first
                                        seed (mem_chain2aln); 0 (default): ref is one strand,
                                        windows are clipped to [0, ref_len) only               */
} bsw_ext_opt_t;

typedef struct bsw_alnreg_t {        /* the mem_alnreg_t fields the extension determines       */
    int64_t rb, re;                  /* [rb, re): reference span                                */
    int32_t qb, qe;                  /* [qb, qe): read span                                     */
    int32_t score;                   /* best local score (last extension's)                     */
    int32_t truesc;                  /* score of the chosen local / to-end ends                 */
    int32_t w;                       /* band actually used (max over both sides)                */
    int32_t seedlen0;                /* seed length                                             */
} bsw_alnreg_t;

void bsw_ext_opt_default(bsw_ext_opt_t *opt);

/* Extend n seeds (read i = reads[read_off[i], read_off[i] + read_len[i]), codes 0..4) against
 * ref[0, ref_len) on the context's devices; scoring = the context's params (a = mat[0]).
 * Reads with seeds[i].len == 0 get a zeroed region.  Blocking; 0 or a BSW_E* code. */
int bsw_extend_seeds(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *ref, int64_t ref_len,
                     const uint8_t *reads, const int64_t *read_off, const int32_t *read_len,
                     const bsw_seed_t *seeds, int32_t n, bsw_alnreg_t *out);

/* Keep ref[0, ref_len) RESIDENT in HBM of every device of the context (replacing any earlier
 * one) for bsw_extend_seeds_device: a 3 Gb genome is ~1% of an MI355X's 288 GB.  Blocking. */
int bsw_set_reference(bsw_ctx_t *ctx, const uint8_t *ref, int64_t ref_len);

/* Device-resident form of bsw_extend_seeds against the resident reference: d_reads, d_read_off,
 * d_read_len, d_seeds and d_out in HBM of the context's first device, `stream` a hipStream_t
 * or NULL.  Job building, band retries and the local / to-end interpretation run on the GPU
 * (bsw_ext_dev.hip); results equal bsw_extend_seeds's.  BSW_E_INVAL without a resident
 * reference.  Both forms validate only seeded reads (seeds[i].len > 0) and return BSW_E_RANGE
 * for the same bad seeds; the device form additionally needs the longest seeded read to
 * satisfy len + 2w + 1 <= BSW_MAX_LEN (its per-read window stride; the host form checks each
 * read's actual window instead).  Returns when d_out holds the regions. */
int bsw_extend_seeds_device(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *d_reads,
                            const int64_t *d_read_off, const int32_t *d_read_len, const bsw_seed_t *d_seeds,
                            int32_t n, bsw_alnreg_t *d_out, void *stream);

/* Batches issued by the last bsw_extend_seeds on ctx: SeqPairs per phase (left, left retry,
 * right, right retry) and the summed DP kernel time. */
typedef struct bsw_ext_stats_t {
    int32_t n_pairs[4];
    float   kernel_ms;               /* DP kernels (HIP events)                                  */
    float   build_ms;                /* host: job lists + code buffers (device form: 0)          */
    float   engine_ms;               /* bsw batches incl. PCIe, plan/sort and kernels (device
                                        form: the whole call)                                    */
    float   interp_ms;               /* host: local / to-end interpretation (device form: 0)     */
} bsw_ext_stats_t;
int bsw_ext_last_stats(bsw_ctx_t *ctx, bsw_ext_stats_t *out);

/* mem_chain2aln over the chains of many reads (upstream's per-read order, batched across reads
 * as mem_chain2aln_across_reads_V2 does).  Seeds are grouped by read
 * (seed_read[k] non-decreasing, indexing read_off / read_len of n_reads reads); within a read,
 * runs of equal seed_chain[k] are its chains, in the order bwa processes them.  Per read: each
 * chain's seeds by score (len * a) descending, ties the later seed first; a seed lying
 * "around" the diagonal of an earlier region of the read (any chain; upstream's containment
 * test with cal_max_gap and the region's band) is SKIPPED unless an extended seed of its own
 * chain, at least 95% as long, overlaps it by >= 1/4 of its length on another diagonal;
 * every other seed is extended exactly as bsw_extend_seeds does.  out[k] = seed k's region
 * (zeroed if skipped), extended[k] = 1 / 0.  Work runs in rounds: round r extends, for every
 * read, the next seed its containment test keeps -- one batch set (LEFT, retries, RIGHT,
 * retries) per round across all reads.  Blocking; 0 or a BSW_E* code. */
int bsw_chain2aln(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *ref, int64_t ref_len,
                  const uint8_t *reads, const int64_t *read_off, const int32_t *read_len, int32_t n_reads,
                  const bsw_seed_t *seeds, const int32_t *seed_read, const int32_t *seed_chain, int32_t n_seeds,
                  bsw_alnreg_t *out, int32_t *extended);

/* The same with the reads RESIDENT in HBM (d_reads on the context's first device, read_off /
 * read_len and the seeds on the host) and the resident reference of bsw_set_reference: the
 * inputs go up once, every per-read step (chain order, containment tests, picks, job arrays)
 * runs on the GPU (csrc/bsw_chain.hip) around the device extension pipeline, one job count per
 * round comes back, the regions come down at the end. */
int bsw_chain2aln_device(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *d_reads,
                         const int64_t *read_off, const int32_t *read_len, int32_t n_reads,
                         const bsw_seed_t *seeds, const int32_t *seed_read, const int32_t *seed_chain,
                         int32_t n_seeds, bsw_alnreg_t *out, int32_t *extended);

/* Fully device-resident form: every array on the context's first device (d_seed_read sorted,
 * as above); regions and flags are written to d_out / d_extended.  No host copies at all --
 * the form a GPU seeding stage (bsw_fmi.h) feeds. */
int bsw_chain2aln_resident(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *d_reads,
                           const int64_t *d_read_off, const int32_t *d_read_len, int32_t n_reads,
                           const bsw_seed_t *d_seeds, const int32_t *d_seed_read, const int32_t *d_seed_chain,
                           int32_t n_seeds, bsw_alnreg_t *d_out, int32_t *d_extended);

typedef struct bsw_chain_stats_t {
    int32_t rounds;                  /* batch rounds of the last bsw_chain2aln(_device)        */
    int32_t n_extended, n_skipped;   /* seeds extended / skipped as contained                  */
    int32_t n_pairs[4];              /* SeqPairs per phase summed over rounds (as ext stats)   */
    float   kernel_ms;               /* DP kernels (HIP events)                                */
    float   ext_ms;                  /* wall time in the rounds' extension calls               */
    float   check_ms;                /* host: containment tests between rounds                 */
    float   prep_ms;                 /* host: per-read chain / seed order                      */
} bsw_chain_stats_t;
int bsw_chain_last_stats(bsw_ctx_t *ctx, bsw_chain_stats_t *out);

#ifdef __cplusplus
}
#endif
#endif /* BSW_EXT_H */
