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

// Same reductions with the row combination done by DPP row_bcast:15 / row_bcast:31 (gfx9 DPP)
// instead of four v_readlane: 6 DPP ops + one v_readlane of lane 63.
__device__ __forceinline__ int wave_max_bc(int x)
{
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x118, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x142, 0xa, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x143, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ int wave_min_bc(int x)
{
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x111, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x112, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x114, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x118, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x142, 0xa, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x143, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(x, 63);
}

// wave_max_bc(xmax) and wave_min_bc(xmin) in one interleaved chain: each DPP step of one
// reduction covers the other's data hazard, so no s_nop sits between dependent DPP ops.
__device__ __forceinline__ void wave_maxmin_bc(int xmax, int xmin, int &omax, int &omin)
{
#define BSW_MM_STEP(ctl, rm)                                                                 \
    xmax = max(xmax, __builtin_amdgcn_update_dpp(INT_MIN, xmax, ctl, rm, 0xf, false));      \
    xmin = min(xmin, __builtin_amdgcn_update_dpp(INT_MAX, xmin, ctl, rm, 0xf, false));
    BSW_MM_STEP(0x111, 0xf) BSW_MM_STEP(0x112, 0xf) BSW_MM_STEP(0x114, 0xf)
    BSW_MM_STEP(0x118, 0xf) BSW_MM_STEP(0x142, 0xa) BSW_MM_STEP(0x143, 0xc)
#undef BSW_MM_STEP
    omax = __builtin_amdgcn_readlane(xmax, 63);
    omin = __builtin_amdgcn_readlane(xmin, 63);
}

typedef const __attribute__((address_space(1))) void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;

}  // namespace bsw
