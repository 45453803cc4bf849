// bsw_mate_k.h -- host-visible launch interface of the mate-rescue kernels (bsw_mate.hip).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "../../include/bsw_seqpair.h"
#include "../../include/bsw_mate.h"

namespace bsw {

struct MateParams {
    int32_t e_del, oe_del, e_ins, oe_ins;
    int32_t maxsc;              // max(mat) >= 1: secondary-hit window te +- ceil(score / maxsc)
    int32_t shift;              // ksw_u8 bias (uint8)(-min(mat)): the u8 pass stops at gmax + shift >= 255
    uint32_t prof[8][2];        // prof[t] = score bytes mat[t][q], q = 0..4; q = 5..7 (padding) -> 0
};

// Job buckets: equal (P, slen) so segment starts are wave-uniform.  0..16: u8 slen 0..16,
// 17..49: i16 slen 0..32.  Kernel classes by ncol = slen * P.
constexpr int kMateBuckets = 50;
constexpr int kMateClasses = 5;
constexpr int kMateNcol[kMateClasses] = {64, 128, 160, 192, 256};
__host__ __device__ inline int mate_class_of_ncol(int ncol)
{
    return ncol <= 64 ? 0 : ncol <= 128 ? 1 : ncol <= 160 ? 2 : ncol <= 192 ? 3 : ncol <= 256 ? 4 : -1;
}
// meta words (device, mirrored to pinned host memory after a prepare)
constexpr int kMateMetaCount = 0;     // [kMateBuckets] jobs per bucket
constexpr int kMateMetaCursor = 64;   // [kMateBuckets] scatter cursors (start, then end)
constexpr int kMateMetaClass = 128;   // [2 * kMateClasses] job-list range of each kernel class
constexpr int kMateMetaTotal = 140;   // job-list length (wave-padded)
constexpr int kMateMetaTmax = 141;    // max target length of the pass's jobs
constexpr int kMateMetaErr = 142;     // nonzero: a job exceeds the supported sizes
constexpr int kMateMetaWords = 144;

// Bucket the jobs of a pass (mode 0: forward over pairs; mode 1: reverse pass of the pairs
// whose forward result in aln needs start positions) into jobs[0, total) (-1 = padding).
// jobs_cap >= n + 64 * kMateBuckets.
hipError_t launch_mate_prepare(const SeqPair *pairs, const bsw_kswr_t *aln, int32_t n, int mode,
                               int32_t *meta, int32_t *jobs, int32_t jobs_cap, hipStream_t s);

// DP kernel of class cls over jobs[j0, j1).  scratch: [row][slot] row maxima (mode 0 only,
// rows >= the pass's max target length, sstride >= total), or null.
hipError_t launch_mate_class(int cls, const MateParams &mp, const SeqPair *pairs, const int32_t *jobs,
                             int32_t j0, int32_t j1, const uint8_t *ref, const uint8_t *qer, bsw_kswr_t *aln,
                             int mode, uint16_t *scratch, int64_t sstride, unsigned long long *cells,
                             hipStream_t s);

}  // namespace bsw
