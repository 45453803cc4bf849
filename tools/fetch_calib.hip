// FETCH_SIZE calibration for the hot kernel's access pattern (tools only; MI355X_MICROARCH.md
// "HBM": calibrate other access widths on a known byte count before trusting an absolute).
//   k_dword_windows : each lane streams its own 300-byte window (75 dwords, windows adjacent
//                     across lanes, as seqBufRef/seqBufQer are read) with 4-byte loads
//   k_lds_dma       : the same windows through global_load_lds_dword (the target stream)
//   k_x4_stream     : coalesced 16 B/lane streaming read (the guide's known 1/2 case, control)
// Each reads BYTES = 2^28 once (256 MiB > L2; run after a 1 GiB flush write to defeat L3) and
// writes 4 bytes per lane.  Run under: rocprofv3 --pmc FETCH_SIZE -- ./tools/fetch_calib
// build: hipcc -O3 --offload-arch=gfx950 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>

constexpr size_t BYTES = size_t(1) << 28;
constexpr int WIN = 300;                          // bytes per lane window

typedef const __attribute__((address_space(1))) void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;

__global__ void k_flush(uint4 *p, size_t n)
{
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4(i, i, i, i);
}

__global__ void k_dword_windows(const uint8_t *buf, uint32_t *out, int nlanes)
{
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nlanes) return;
    const uint32_t *w = (const uint32_t *)(buf + (size_t)g * WIN);
    uint32_t acc = 0;
#pragma unroll 5
    for (int k = 0; k < WIN / 4; ++k) acc += w[k] * (k + 1);
    out[g] = acc;
}

__global__ void k_lds_dma(const uint8_t *buf, uint32_t *out, int nlanes)
{
    __shared__ uint32_t s[WIN / 4][256];
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t *w = (const uint32_t *)(buf + (size_t)min(g, nlanes - 1) * WIN);
    for (int k = 0; k < WIN / 4; ++k)
        __builtin_amdgcn_global_load_lds((gptr_t)(w + k), (lptr_t)&s[k][threadIdx.x & ~63], 4, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    uint32_t acc = 0;
    for (int k = 0; k < WIN / 4; ++k) acc += s[k][threadIdx.x] * (k + 1);
    if (g < nlanes) out[g] = acc;
}

__global__ void k_x4_stream(const uint4 *buf, uint32_t *out, size_t n4)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = buf[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main()
{
    uint8_t *buf; uint32_t *out; uint4 *fl;
    const int nlanes = (int)(BYTES / WIN);
    const int x4_grid = 8192;
    // out holds one word per lane of every kernel: max(nlanes, x4_grid * 256) entries
    const size_t nout = std::max((size_t)nlanes, (size_t)x4_grid * 256);
    if (hipMalloc(&buf, BYTES + 4096) != hipSuccess || hipMalloc(&out, sizeof(uint32_t) * nout) != hipSuccess ||
        hipMalloc(&fl, size_t(1) << 30) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    (void)hipMemset(buf, 1, BYTES);
    const dim3 b(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_flush, dim3(4096), b, 0, 0, fl, (size_t(1) << 30) / 16);
        hipLaunchKernelGGL(k_dword_windows, dim3((nlanes + 255) / 256), b, 0, 0, buf, out, nlanes);
        hipLaunchKernelGGL(k_flush, dim3(4096), b, 0, 0, fl, (size_t(1) << 30) / 16);
        hipLaunchKernelGGL(k_lds_dma, dim3((nlanes + 255) / 256), b, 0, 0, buf, out, nlanes);
        hipLaunchKernelGGL(k_flush, dim3(4096), b, 0, 0, fl, (size_t(1) << 30) / 16);
        hipLaunchKernelGGL(k_x4_stream, dim3(x4_grid), b, 0, 0, (const uint4 *)buf, out, BYTES / 16);
    }
    (void)hipDeviceSynchronize();
    printf("known bytes read per launch: %zu (windows: %d lanes x %d B); writes: %zu / %zu\n", BYTES,
           nlanes, WIN, sizeof(uint32_t) * (size_t)nlanes, sizeof(uint32_t) * (size_t)x4_grid * 256);
    return 0;
}
