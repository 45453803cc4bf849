/*
 * bsw_fmi.h -- FM-index SMEM seeding on the GPU (second half).
 *
 * Replaces the seeding half of upstream bwa-mem2's per-read pipeline (the reference names it
 * as 80% of runtime, PHASE4_SEEDING_ANALYSIS.md:32-66): FMI_search::backwardExt /
 * getSMEMsOnePosOneThread / getSMEMsAllPosOneThread / bwtSeedStrategyAllPosOneThread in
 * src/FMI_search.cpp and mem_collect_intv in src/bwamem.cpp [UPSTREAM-RECALL; the reference
 * holds no source of them].  Semantics = lh3/bwa's bwt_smem1a + bwt_seed_strategy1 +
 * mem_collect_intv, which bwa-mem2 documents as output-identical:
 *
 *   pass 1  x = 0; while x < len: x = smem1(x, min_intv = 1) keeping SMEMs of >= min_seed_len
 *   pass 2  for every pass-1 SMEM of length >= min_seed_len * split_factor (+.499, truncated)
 *           and occurrence s <= split_width: smem1((start + end) >> 1, min_intv = s + 1)
 *   pass 3  (max_mem_intv > 0) LAST-like seeds: from x, the shortest forward match of length
 *           >= min_seed_len + 1 with fewer than max_mem_intv occurrences
 *   then sorted by info (qbeg << 32 | qend); ties (upstream's introsort leaves them unordered)
 *   by k, s, l.  No parity gap: equal info is the same read substring, whose SA interval and
 *   reverse-complement row are unique, so tied records are identical and every order of them
 *   is the same sequence (tests/test_fmi.py::test_tied_intervals_are_identical).
 *
 * Scope of the seeding -> chaining front end (bsw_mem_chain_device, bsw_chain2aln_resident):
 *   - ONE reference sequence (a bntseq with a single contig).  Upstream also drops seeds that
 *     span two contigs (bns_intv2rid < 0), refuses chain merges across contigs (seed rid !=
 *     chain rid) and clips extension windows to the contig (bns_fetch_seq); here the only
 *     boundary is the forward / reverse strand one (l_pac).  A multi-sequence genome (GRCh38)
 *     must be given as one concatenated sequence, and seeds / chains / windows that cross its
 *     contig joins are NOT filtered as upstream filters them.
 *   - reads shorter than ~720 bp.  Upstream's mem_align1_core runs mem_flt_chained_seeds
 *     between chaining and extension; it returns at once while MEM_MINSC_COEF * ln(l) >
 *     MEM_SEEDSW_COEF * l (5.5 ln l > 0.05 l: l <= 720 with min_chain_weight 0) and is not
 *     restated here, so longer reads' seeds (hence regions) may differ from upstream.
 *
 * Index (built on the host below 64 Mb, on the GPU above; resident in HBM): T = ref +
 * reverse-complement(ref), the BWT of T$ with the sentinel kept, count[c] = 1 + #{bases < c},
 * occurrence counts in 64-base blocks of 64 bytes (4 x uint32 -- or, in the wide layout, 4 x
 * uint64 -- counts + 4 x uint64 one-hot masks: one block load per Occ query), the full suffix
 * array as uint32 (|T| + 1 < 2^32) or uint64 (the wide layout a 3 Gb genome's 6 G rows need).  Intervals are bwa-mem2's:
 * [k, k + s) 0-based over the n + 1 rows of T$, l = k of the reverse-complement string.
 * Reference bases must be 0..3 (ambiguous bases replaced beforehand, as bwa's .pac does);
 * read bases 0..4 (4 = N ends every match).
 */
#ifndef BSW_FMI_H
#define BSW_FMI_H

#include <stdint.h>
#include "bsw.h"
#include "bsw_ext.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bsw_fmi bsw_fmi_t;

/* bwa's bwtintv_t: x[0] = k, x[1] = l, x[2] = s (occurrences), info = qbeg << 32 | qend */
typedef struct bsw_bwtintv_t {
    uint64_t x[3];
    uint64_t info;
} bsw_bwtintv_t;

typedef struct bsw_mem_opt_t {       /* the mem_opt_t fields seeding reads                        */
    int32_t min_seed_len;            /* bwa -k (19)                                               */
    int32_t split_width;             /* re-seed SMEMs with at most this many occurrences (10)     */
    int32_t max_mem_intv;            /* pass-3 occurrence bound; 0 disables pass 3 (20)           */
    float   split_factor;            /* bwa -r (1.5)                                              */
} bsw_mem_opt_t;

typedef struct bsw_fmi_info_t {
    int64_t n;                       /* |T| = 2 * ref_len (the BWT has n + 1 rows)                */
    int64_t sentinel;                /* BWT row holding '$' (SA = 0)                              */
    int64_t count[5];                /* count[c] = 1 + #{T[i] < c}                                */
    int64_t device_bytes;            /* HBM held by the resident index                            */
    float   build_s;                 /* host build time (suffix array + BWT + blocks)             */
} bsw_fmi_info_t;

void bsw_mem_opt_default(bsw_mem_opt_t *opt);

/* Build the FM-index of ref[0, ref_len) -- below 64 Mb on the host (prefix-doubling suffix array
 * over 27-base keys), else on the GPU (bsw_fmi_build2) -- and keep it resident on HIP device
 * `device` (device < 0: host-only index -- suffix array,
 * BWT and counts for inspection; seeding calls on it return BSW_E_NODEV).  Blocking.
 * BSW_E_INVAL for a base > 3.  (Host-only indexes are narrow: BSW_E_RANGE past 2^32 rows.) */
int  bsw_fmi_build(const uint8_t *ref, int64_t ref_len, int device, bsw_fmi_t **out);
/* The same with builder flags: BSW_FMI_GPU_BUILD builds on the GPU (bucketed radix sort of 27-base
 * keys in HBM, csrc/bsw_fmi_build.hip), BSW_FMI_WIDE keeps 64-bit rows / counts / suffix array.
 * bsw_fmi_build picks them itself: references of >= 64 Mb build on the GPU, and a two-strand text
 * of >= 2^32 - 1 rows (a ~2.1 Gb genome or larger, e.g. GRCh38's 3.1 Gb) needs the wide layout:
 * 8 B of suffix array + 1 B of occurrence blocks + 1 B of BWT codes per text position, ~60 GB of
 * HBM for 3 Gb (ABI version 5). */
/* Unless BSW_FMI_NO_TEXT is given the index also keeps the two-strand text (1 B per position) and
 * the inverse suffix array (4 / 8 B per row) in HBM: once an interval is down to one occurrence
 * the SMEM walk extends it by comparing read and text directly instead of one dependent
 * occurrence-block load per base (outputs identical). */
/* BSW_FMI_PLAIN_ENT (tests, ABI 8): the wide index's SMEM walk keeps its interval vectors in plain
 * 32-B entries even when every value fits the packed 16-B form (the fallback of indexes past 2^40
 * rows or with a single base's count past 2^32), so that path is exercised at small sizes. */
enum { BSW_FMI_GPU_BUILD = 1, BSW_FMI_WIDE = 2, BSW_FMI_NO_TEXT = 4, BSW_FMI_PLAIN_ENT = 8 };
int  bsw_fmi_build2(const uint8_t *ref, int64_t ref_len, int device, int flags, bsw_fmi_t **out);
void bsw_fmi_destroy(bsw_fmi_t *fmi);
int  bsw_fmi_get_info(const bsw_fmi_t *fmi, bsw_fmi_info_t *out);
/* Host copies of the suffix array (n + 1 entries) and the BWT (n + 1 codes, 4 = '$'). */
int  bsw_fmi_copy_sa(const bsw_fmi_t *fmi, int64_t *sa);
int  bsw_fmi_copy_bwt(const bsw_fmi_t *fmi, uint8_t *bwt);

/* mem_collect_intv for n reads (read i = reads[read_off[i], read_off[i] + read_len[i]), codes
 * 0..4): up to `cap` intervals of read i at mems[i * cap], their number in n_mems[i].  If some
 * read has more than cap, its n_mems is > cap (a lower bound of the true count: re-seeding only
 * sees the SMEMs that were stored), its intervals are incomplete, and the call returns
 * BSW_E_RANGE; reads with n_mems <= cap are exact.  Host buffers; blocking. */
int  bsw_mem_collect_intv(bsw_fmi_t *fmi, const bsw_mem_opt_t *opt, const uint8_t *reads,
                          const int64_t *read_off, const int32_t *read_len, int32_t n,
                          bsw_bwtintv_t *mems, int32_t cap, int32_t *n_mems);

/* Device-resident form (all pointers in HBM of the index's device; max_len >= every read
 * length bounds the per-read scratch).  `stream` a hipStream_t or NULL.  Returns when the
 * results are in HBM; BSW_E_RANGE as above (the overflow flag is read back). */
int  bsw_mem_collect_intv_device(bsw_fmi_t *fmi, const bsw_mem_opt_t *opt, const uint8_t *d_reads,
                                 const int64_t *d_read_off, const int32_t *d_read_len, int32_t n,
                                 int32_t max_len, bsw_bwtintv_t *d_mems, int32_t cap,
                                 int32_t *d_n_mems, void *stream);

/* bwt_sa over device arrays: d_pos[i] = SA[d_k[i]] (text position of BWT row k; positions
 * >= ref_len lie on the reverse strand, as bns_depos reads them).  Rows > n give -1. */
int  bsw_fmi_sa_device(bsw_fmi_t *fmi, const uint64_t *d_k, int64_t n, int64_t *d_pos, void *stream);

/* Self-check of a resident index on its device: the occurrence blocks' running counts chain and
 * end at count[], the suffix array is a permutation of [0, n], and every row's LF step lands on
 * the suffix one position earlier (SA[LF(r)] = SA[r] - 1).  *bad = violations (0 = consistent);
 * ~1 s for a 3 Gb genome.  BSW_E_NODEV for a host-only index. */
int  bsw_fmi_check(bsw_fmi_t *fmi, int64_t *bad);

/* The last seeding call's SMEM kernel time (HIP events). */
int  bsw_fmi_last_kernel_ms(const bsw_fmi_t *fmi, float *ms);

/* ---------------------------------------------------------------- seeds -> chains
 * mem_chain + mem_chain_flt (bwa src/bwamem.c, kept by bwa-mem2's src/bwamem.cpp;
 * [UPSTREAM-RECALL]: the reference holds no source of them), per read over its
 * mem_collect_intv intervals, on the GPU (csrc/bsw_memchain.hip):
 *   for each interval (in info order), step = s > max_occ ? s / max_occ : 1, and for
 *   k = 0, 1 step, ... while k < s and fewer than max_occ taken: seed = (rbeg = SA[k0 + k],
 *   qbeg, len = score = qend - qbeg); a seed across the forward / reverse boundary l_pac is
 *   dropped (bns_intv2rid < 0); otherwise the chain with the largest start <= rbeg (kbtree
 *   kb_intervalp) absorbs it when test_and_merge says so (contained seed, or same strand and
 *   |diagonal drift| <= w with gaps < max_chain_gap from the chain's last seed), else it
 *   starts a new chain.  Chains in start order, then mem_chain_flt: weight = min(query, ref)
 *   coverage of the chain's seeds; chains below min_chain_weight dropped; sorted by weight
 *   descending (klib ks_introsort, as upstream -- ties in its order); a chain significantly
 *   overlapping (>= mask_level of the shorter, shorter < max_chain_gap) a kept heavier one is
 *   dropped when lighter than drop_ratio of it by >= 2 * min_seed_len, else kept as
 *   secondary; max_chain_extend bounds the secondaries.
 * Output = the input bsw_chain2aln_resident takes: seeds grouped by read (seed_read
 * ascending), each read's chains as runs of seed_chain (0, 1, ... in processing order), each
 * chain's seeds in chain order.  Duplicate chain starts follow a single-leaf kbtree (a new
 * chain goes right after the first chain of equal start). */
typedef struct bsw_chain_opt_t {
    int32_t max_occ;                 /* bwa -c: occurrences sampled per interval (500)            */
    int32_t w;                       /* bwa -w: band of test_and_merge (100)                      */
    int32_t max_chain_gap;           /* 10000                                                     */
    int32_t min_chain_weight;        /* bwa -W (0)                                                */
    int32_t min_seed_len;            /* bwa -k (19): mem_chain_flt's "much lighter" margin / 2    */
    int32_t max_chain_extend;        /* secondaries extended at most (1 << 30)                    */
    float   drop_ratio;              /* bwa -D (0.5)                                              */
    float   mask_level;              /* 0.5                                                       */
} bsw_chain_opt_t;

void bsw_chain_opt_default(bsw_chain_opt_t *opt);

/* Seeds and chains of n_reads reads from their intervals (d_mems[i * cap + t], t < d_n_mems[i],
 * as bsw_mem_collect_intv_device leaves them) against the index's suffix array, all device
 * arrays on the index's device.  Writes at most seed_cap seeds (d_seeds, d_seed_read,
 * d_seed_chain) and their number to *n_seeds; BSW_E_RANGE (with *n_seeds = the number needed)
 * when seed_cap is too small.  Blocking. */
int  bsw_mem_chain_device(bsw_fmi_t *fmi, const bsw_chain_opt_t *opt, const int32_t *d_read_len, int32_t n_reads,
                          const bsw_bwtintv_t *d_mems, int32_t cap, const int32_t *d_n_mems, bsw_seed_t *d_seeds,
                          int32_t *d_seed_read, int32_t *d_seed_chain, int64_t seed_cap, int64_t *n_seeds,
                          void *stream);

#ifdef __cplusplus
}
#endif
#endif /* BSW_FMI_H */
