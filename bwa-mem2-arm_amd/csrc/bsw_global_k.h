// bsw_global_k.h -- host-visible launch interface of the global-alignment kernels (bsw_global.hip).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "../../include/bsw_seqpair.h"
#include "../../include/bsw_global.h"

namespace bsw {

struct GlobParams {
    int32_t o_del, e_del, o_ins, e_ins, oe_del, oe_ins;
    int32_t maxabs;             // max |mat| -- the int16 safety bound of the register kernel
    uint32_t prof[8][2];        // prof[t] = score bytes mat[t][q], q = 0..4; q = 5..7 score as N
    int8_t mat[25];
    int8_t prefer_band;         // route band-eligible jobs to the band kernel (BSW_OPT_GLOB_BAND)
};

// Job classes: band-coordinate register kernel (int32 cells, 2w + 2 <= BW slots), column
// register kernel for qlen <= QMAX (int16-safe scores), then the int32 wide kernel (eh row in
// HBM).  Routing in glob_class (bsw_global.hip).
constexpr int kGlobBandClasses = 5;
constexpr int kGlobBandW[kGlobBandClasses] = {32, 48, 64, 80, 96};
constexpr int kGlobLaneClasses = 5;
constexpr int kGlobQmax[kGlobLaneClasses] = {32, 64, 96, 128, 160};
constexpr int kGlobLane0 = kGlobBandClasses;                       // first column class
constexpr int kGlobWideClass = kGlobLane0 + kGlobLaneClasses;
constexpr int kGlobClasses = kGlobWideClass + 1;
// meta words: counts, max tlen, max w, max qlen per class; error flag
// per slot (kGMetaSpread slots, each in its own lines; the host reduces them): counts, max
// tlen, max w, max qlen per class, error flag
constexpr int kGMetaCount = 0, kGMetaTmax = 16, kGMetaWmax = 32, kGMetaQmax = 48, kGMetaErr = 64;
constexpr int kGMetaWordsPerSlot = 80;
constexpr int kGMetaSpread = 16;
constexpr int kGMetaWords = kGMetaWordsPerSlot * kGMetaSpread;
static_assert(kGlobClasses <= 16, "meta layout");
constexpr int kGlobKeyBits = 32;

// Traceback-matrix dwords per row of a class's waves (8 nibbles per dword): the row window
// starting at dword max(i - wmax, 0) >> 3 covers every lane's band [max(i - w, 0), i + w].
// (Band classes: one dword per 8 slots of the fixed band window, BW / 8.)
inline int glob_cap_dw(int cls, int qmax, int wmax)
{
    if (cls < kGlobBandClasses) return kGlobBandW[cls] / 8;
    const int band = ((2 * wmax) >> 3) + 2;
    const int full = cls < kGlobWideClass ? kGlobQmax[cls - kGlobLane0] / 8 : (qmax + 7) / 8 + 1;
    return band < full ? band : full;
}

// Per job: class + scheduling key (class, w desc, qlen desc, tlen desc); meta per class.
hipError_t launch_glob_plan(const SeqPair *pairs, int32_t n, const GlobParams &gp, uint32_t *keys,
                            int32_t *vals, int32_t *meta, hipStream_t s);

// DP + traceback of class cls over jobs order[0, n).  z: traceback matrix, zstride uint32 per
// wave (>= max tlen * cap_dw * 64), null for scores only; ehs: int32 row scratch of the wide
// class, (max qlen + 1) * n int2.
// tb_dw > 0 (column classes only): narrow traceback window -- each lane stores per row only tb_dw
// dwords around its diagonal corridor (glob_lane_kernel); jobs whose path leaves it are appended
// to retry[1..] (count in retry[0]) for a full-window rerun.  Row stride of z: tb_dw or cap_dw.
hipError_t launch_glob_class(int cls, const GlobParams &gp, SeqPair *pairs, const int32_t *order, int32_t n,
                             const uint8_t *ref, const uint8_t *qer, uint32_t *z, int64_t zstride,
                             int32_t cap_dw, int2 *ehs, uint32_t *cigar, int32_t stride, int32_t *n_cigar,
                             unsigned long long *cells, hipStream_t s, int32_t tb_dw = 0, int32_t *retry = nullptr);

}  // namespace bsw
