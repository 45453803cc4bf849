// Probe (GPU box): can helper-stream kernels run beside a grid that fills every VGPR of its CUs?
// A "waiter" grid of ~250-VGPR waves (the persistent DP kernel's footprint) runs on a CU-masked DP
// stream and polls a flag (relaxed agent loads, 2-s bound); on the helper stream (the
// complementary CU mask) an optional 256-thread kernel runs first, then a one-thread setter raises
// the flag.  Reports how long the helper stream took -- ~0 when the masks keep the two apart, ~2 s
// when the helper's kernels wait for the waiters to give up.  Run with few streams, then after
// PROBE_STREAMS more streams (every third high priority) each ran a kernel: the library's state.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

__global__ __launch_bounds__(64) void waiter(int *flag, int *out)
{
    // ~250 VGPRs live across the poll (as pq_kernel): the compiler must allocate them all
    asm volatile("" ::: "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210",
                 "v211", "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222",
                 "v223", "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234",
                 "v235", "v236", "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246",
                 "v247", "v248", "v249");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int v = 0;
    for (;;) {
        v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;
        __builtin_amdgcn_s_sleep(8);
    }
    if (threadIdx.x == 0) {
        atomicMax(out, (int)((__builtin_amdgcn_s_memrealtime() - t0) / 100));
        if (!v) atomicOr(out + 1, 1);
    }
}
__global__ void busy256(int *x, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = i * 3;
}
__global__ void setter(int *flag)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static int run(const char *tag, const uint32_t *hmask, int ncu, bool big)
{
    const int nw = (ncu + 31) / 32;
    uint32_t hm[32] = {}, dm[32] = {};
    int nres = 0;
    for (int c = 0; c < ncu; ++c) {
        const bool r = (hmask[c / 32] >> (c % 32)) & 1;
        nres += r;
        (r ? hm : dm)[c / 32] |= 1u << (c % 32);
    }
    hipStream_t h, d;
    CK(hipExtStreamCreateWithCUMask(&h, (uint32_t)nw, hm));
    CK(hipExtStreamCreateWithCUMask(&d, (uint32_t)nw, dm));
    int *flag, *out, *scratch;
    CK(hipMalloc(&flag, 4)); CK(hipMalloc(&out, 8)); CK(hipMalloc(&scratch, (1 << 22) * 4));
    CK(hipMemset(flag, 0, 4)); CK(hipMemset(out, 0, 8));
    CK(hipDeviceSynchronize());
    const int grid = 8 * (ncu - nres);
    hipLaunchKernelGGL(waiter, dim3(grid), dim3(64), 0, d, flag, out);
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    const auto t0 = std::chrono::steady_clock::now();
    if (big) hipLaunchKernelGGL(busy256, dim3((1 << 22) / 256), dim3(256), 0, h, scratch, 1 << 22);
    hipLaunchKernelGGL(setter, dim3(1), dim3(64), 0, h, flag);
    CK(hipStreamSynchronize(h));
    const double hms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    CK(hipStreamSynchronize(d));
    int o[2];
    CK(hipMemcpy(o, out, 8, hipMemcpyDeviceToHost));
    printf("%-44s reserve %3d, grid %5d: helper stream %8.2f ms; waiters %7d us, timed out %d\n", tag, nres, grid, hms,
           o[0], o[1]);
    CK(hipFree(flag)); CK(hipFree(out)); CK(hipFree(scratch));
    CK(hipStreamDestroy(h)); CK(hipStreamDestroy(d));
    return 0;
}

int main()
{
    CK(hipSetDevice(0));
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int ncu = pr.multiProcessorCount;
    printf("%s, %d CUs\n", pr.gcnArchName, ncu);
    uint32_t m1[32] = {}, m2[32] = {};
    for (int w = 0; w < 8; ++w) m1[w] = 1u;       // bit 0 of each 32-CU word
    m2[0] = 0xffu;                                // CUs 0-7
    if (run("bit 0 of each word, setter only", m1, ncu, false)) return 1;
    if (run("bit 0 of each word, 256-thread kernel first", m1, ncu, true)) return 1;
    if (run("CUs 0-7, 256-thread kernel first", m2, ncu, true)) return 1;
    const int ns = getenv("PROBE_STREAMS") ? atoi(getenv("PROBE_STREAMS")) : 24;
    std::vector<hipStream_t> extra;
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    int *x;
    CK(hipMalloc(&x, 1 << 20));
    for (int k = 0; k < ns; ++k) {
        hipStream_t t;
        if (k % 3 == 2) CK(hipStreamCreateWithPriority(&t, hipStreamNonBlocking, hi));
        else CK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
        hipLaunchKernelGGL(busy256, dim3(16), dim3(256), 0, t, x, 4096);
        extra.push_back(t);
    }
    CK(hipDeviceSynchronize());
    printf("-- after %d more streams (every third high priority) each ran a kernel:\n", ns);
    if (run("bit 0 of each word, setter only", m1, ncu, false)) return 1;
    if (run("bit 0 of each word, 256-thread kernel first", m1, ncu, true)) return 1;
    if (run("CUs 0-7, 256-thread kernel first", m2, ncu, true)) return 1;
    return 0;
}
