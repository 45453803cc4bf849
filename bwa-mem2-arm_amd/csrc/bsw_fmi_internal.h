// bsw_fmi_internal.h -- the resident index as the other device stages see it (not installed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <mutex>
#include "../../include/bsw_fmi.h"

namespace bsw {
// One 64-byte occurrence block per 64 BWT rows, two widths: narrow (|T| + 1 < 2^32: 32-bit
// counts) and wide (a 3 Gb genome's 6 G rows: 64-bit counts).  The bit masks sit at byte 32 in
// both.  cnt[c] = #c in rows [0, 64b); bit y of bits[c] = row 64b + y holds c.
struct alignas(64) FmiBlock {
    uint32_t cnt[4];
    uint32_t pad[4];
    uint64_t bits[4];
};
struct alignas(64) FmiBlockW {
    uint64_t cnt[4];
    uint64_t bits[4];
};
static_assert(sizeof(FmiBlock) == 64 && sizeof(FmiBlockW) == 64, "one 64-byte block per 64 rows");

// Device buffers of an index built on the GPU (bsw_fmi_build.hip); the bsw_fmi_t owns them.
struct GpuIndex {
    void *d_sa = nullptr;            // SA of T$: uint32_t (narrow) or uint64_t (wide), n + 1 rows
    void *d_blk = nullptr;           // FmiBlock or FmiBlockW, n / 64 + 1 blocks
    uint8_t *d_bwt = nullptr;        // BWT codes (4 = '$'), n + 1 rows
    int64_t n = 0, sentinel = 0;
    int64_t count[5] = {0, 0, 0, 0, 0};
    int64_t tie_groups = 0;          // suffix groups equal on 27 bases, resolved by comparison
};
// Build the index of ref (codes 0..3) on `device`: T = ref + revcomp(ref) made in HBM, the
// suffix array by bucketing (first 3 bases) + per-bucket radix sort of 27-base keys + direct
// comparison of the remaining tie groups, then BWT and occurrence blocks.  Blocking.
int fmi_build_gpu(const uint8_t *ref, int64_t ref_len, int device, bool wide, GpuIndex *out);
// Invariants of a resident index: block counts chain, SA a permutation, LF(r) = SA^-1[SA[r] - 1];
// *bad = number of violations (0: consistent).  d_bwt: the BWT codes on the device.
int fmi_check_gpu(int device, bool wide, const void *d_sa, const uint8_t *d_bwt, const void *d_blk, int64_t n,
                  const int64_t *count, int64_t *bad);

struct FmiView {
    int device;
    const void *d_sa;                // suffix array of T$ (n + 1 rows): uint32_t or uint64_t
    bool sa64;
    int64_t n;                       // |T| = 2 * l_pac
    int64_t l_pac;                   // forward-strand length
    hipStream_t stream;              // the index's own stream
    std::mutex *mu;                  // one call at a time per index
};
// BSW_E_NODEV for a host-only index
int fmi_view(bsw_fmi_t *f, FmiView *out);
}  // namespace bsw
