// bsw_wave.h -- wave-level helpers shared by the gfx950 DP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <limits.h>

namespace bsw {

// Wave-uniform max / min over all 64 lanes (exec must be full): DPP row_shr scan inside
// each 16-lane row, then the four row results via v_readlane.
__device__ __forceinline__ int wave_max(int x)
{
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x118, 0xf, 0xf, false));
    int a = __builtin_amdgcn_readlane(x, 15), b = __builtin_amdgcn_readlane(x, 31);
    int c = __builtin_amdgcn_readlane(x, 47), d = __builtin_amdgcn_readlane(x, 63);
    return max(max(a, b), max(c, d));
}
__device__ __forceinline__ int wave_min(int x)
{
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x111, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x112, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x114, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x118, 0xf, 0xf, false));
    int a = __builtin_amdgcn_readlane(x, 15), b = __builtin_amdgcn_readlane(x, 31);
    int c = __builtin_amdgcn_readlane(x, 47), d = __builtin_amdgcn_readlane(x, 63);
    return min(min(a, b), min(c, d));
}

typedef const __attribute__((address_space(1))) void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;

}  // namespace bsw
