// bsw_kernels.h -- host-visible launch interface of the seed-extension DP kernels (gfx950).
//
// Kernel families:
//   lane kernel  : one LANE per SeqPair, the whole DP row of the pair (eh[0..qlen], packed
//                  {h:16, e:16} per column) held in VGPRs; 64 pairs per wavefront advance
//                  through their target rows in lock-step.  qlen <= QMAX (template), int16 cells.
//   pc kernel    : one SeqPair per lane, the DP row as an H plane and an E plane packed two
//                  columns per VGPR, column-independent steps as v_pk_* (bsw_pc.hip);
//                  bwa-style scoring, scores < 256.  The default 8-bit-regime kernel.
//   wide kernel  : one lane per pair, eh row in HBM scratch, int32 cells; any length.
//                  Used for qlen > QMAX or scores that could overflow int16.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "../../include/bsw_seqpair.h"

namespace bsw {

// Scoring constants as the kernels consume them.
struct KParams {
    int32_t o_del, e_del, o_ins, e_ins;
    int32_t zdrop, end_bonus;
    int32_t maxsc;              // max(0, max(mat)) -- A.2 band cap and the M-gate bound
    int32_t pk_ok;              // scoring fits the packed-column kernel (match 1, mismatch -b,
                                //   N -1, symmetric gaps); set by the host, see bsw_pc.hip
    uint32_t prof[8][2];        // prof[t] = 8 score bytes mat[t][q], q = 0..7 (q>4 -> ambig)
    int8_t mat[25];
    int8_t kern8;               // host: 8-bit-regime pairs -> 1 packed-column kernel, 0 lane
                                //   kernel (BSW_OPT_KERNEL8)
    int8_t keymode;             // host: plan sort-key variant (BSW_OPT_SORTKEY)
    int8_t fork;                // host: class launches fork over side streams (BSW_OPT_FORK)
    int8_t misroute;            // host, tests only: every pair to the QMAX=32 lane class
                                //   (BSW_OPT_TEST_MISROUTE: trips the kernels' range guard)
    int8_t long_route;          // host: queries past 160 columns -> 1 wave kernel (default),
                                //   0 wide kernel, 2 every qualifying pair to the wave kernel
                                //   (BSW_OPT_LONG)
    int8_t group_kernel;        // host: small batches on the row-group kernel (bsw_gq.hip,
                                //   BSW_OPT_GROUP_KERNEL)
    int32_t mid_batch;          // host: calls / chunks of (small_batch, mid_batch] pairs run on
                                //   the quad row-group kernel (BSW_OPT_MID_BATCH, 0 = off)
    int32_t small_batch;        // host: calls / chunks of at most this many pairs run every
                                //   qualifying pair on the wave kernel (latency, not
                                //   throughput, bounds them; BSW_OPT_SMALL_BATCH, 0 = off)
    int32_t gq32_max;           // host: batches of at most this many pairs (within small_batch)
                                //   take the row-group kernel's 32-lane latency form
                                //   (BSW_OPT_GQ32_MAX, default 2048)
};

// The kernels' input fields of a SeqPair (staged without the caller bookkeeping and outputs):
// 20 B per pair in the host pipeline's staging buffers and the packed wire form (bsw.h).
struct PairIn {
    int32_t idr, idq, len1, len2, h0;
};
static_assert(sizeof(PairIn) == 20, "PairIn");

// qlen limit of the register-resident kernel instantiations.
constexpr int kLaneQmax[] = {32, 64, 96, 128, 160};
constexpr int kLaneQmaxMax = 160;

// Launch the lane kernel for pairs order[0..n) (indices into pairs).  qlen of every pair
// must be <= qmax (one of kLaneQmax) and h0 + maxsc*min(len1,len2) < 32768.
hipError_t launch_lane_kernel(int qmax, const KParams &kp, int32_t w, SeqPair *pairs,
                              const int32_t *order, int32_t n, const uint8_t *ref,
                              const uint8_t *qer, int32_t *err, hipStream_t s);

// Packed-column lane kernel (bsw_pc.hip): kp.pk_ok scoring, qlen < qmax (strictly: slot qlen
// must fall inside a 4-column group), h0 + min(len1, len2) <= 255; 64 pairs per wave.
hipError_t launch_pc_kernel(int qmax, const KParams &kp, int32_t w, SeqPair *pairs,
                            const int32_t *order, int32_t n, const uint8_t *ref,
                            const uint8_t *qer, int32_t *err, hipStream_t s);

// Wave-per-alignment band kernel (bsw_wv.hip): one SeqPair per wavefront, the row spread over
// the 64 lanes as a sliding window of 64 * cols absolute columns (cols = 4, 8 or 16).  Needs
// max(mat) == 1, qlen <= kWvQmax, 2 * wl + cols + 2 <= 64 * cols (wl = the pair's band cap) and
// int16-safe values (h0 + min(qlen, tlen) + e_ins * (qlen + 1) < 30000, e_ins * qlen < 2700).
constexpr int kWvQmax = 4096;
hipError_t launch_wv_kernel(int cols, const KParams &kp, int32_t w, SeqPair *pairs, const int32_t *order,
                            int32_t n, const uint8_t *ref, const uint8_t *qer, int32_t *err, hipStream_t s);

// Small-batch row-group kernel (bsw_gq.hip): one group of gs lanes per SeqPair -- gs = 16 (one
// DPP row; cols 4, 6, 8 or 10 per lane) for small batches, gs = 4 (a quad; cols 16, 24, 32 or 40)
// for medium ones -- queries up to gs * cols, 64 / gs pairs per wave, no plan or sort needed.
// Pairs outside its contract (gq_pair_ok) are skipped and set *flag (or *err when flag is
// null).  order may be null (pair k = slot k).
hipError_t launch_gq_kernel(int gs, int cols, const KParams &kp, int32_t w, SeqPair *pairs, const int32_t *order,
                            int32_t n, const uint8_t *ref, const uint8_t *qer, int32_t *err, int32_t *flag,
                            int32_t *out24, hipStream_t s);
int gq_cols_for(int max_qlen, int gs);                 // -1 past 160 columns
bool gq_pair_ok(const KParams &kp, int qlen, int tlen, int h0, int gs);   // host-side contract check

// Wide kernel: any qlen/tlen, int32 cells, eh scratch of n * (max_qlen + 2) int2 in HBM.
hipError_t launch_wide_kernel(const KParams &kp, int32_t w, SeqPair *pairs,
                              const int32_t *order, int32_t n, const uint8_t *ref,
                              const uint8_t *qer, int2 *scratch, int32_t scratch_stride,
                              hipStream_t s);

}  // namespace bsw
