// bsw_fmi_internal.h -- the resident index as the other device stages see it (not installed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <mutex>
#include "../../include/bsw_fmi.h"

namespace bsw {
struct FmiView {
    int device;
    const uint32_t *d_sa;            // suffix array of T$ (n + 1 rows)
    int64_t n;                       // |T| = 2 * l_pac
    int64_t l_pac;                   // forward-strand length
    hipStream_t stream;              // the index's own stream
    std::mutex *mu;                  // one call at a time per index
};
// BSW_E_NODEV for a host-only index
int fmi_view(bsw_fmi_t *f, FmiView *out);
}  // namespace bsw
