// Cycle cost of the real packed-kernel group (bsw::pk_group from bsw_pk.hip) in a loop, one wave
// per SIMD, fast and masked paths (tools only).
// build: hipcc -O3 --offload-arch=gfx950 -Iinclude -o tools/pk_group_bench tools/pk_group_bench.hip
#include "../bwa-mem2-arm_amd/csrc/bsw_pk.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
#define ITERS 512

template <int MODE>   // 0: fast path, 1: masked path, 2: skip
__global__ __launch_bounds__(256, 1) void kgrp(unsigned long long *out, int seed)
{
    uint32_t hh[9], ee[8], qp[4];
#pragma unroll
    for (int k = 0; k < 9; ++k) hh[k] = (threadIdx.x * 7 + k * 13 + seed) & 0x007f007fu;
#pragma unroll
    for (int k = 0; k < 8; ++k) ee[k] = (threadIdx.x * 3 + k) & 0x001f001fu;
#pragma unroll
    for (int k = 0; k < 4; ++k) qp[k] = 0x01020300u + k + seed;
    uint32_t hc = 5, hg = 5, f = 0, key = 0, lp = 0;
    const uint32_t tw = 0x0c010c02u, tl = 0xfcfcfc01u, th = 0xffffffffu;
    const uint32_t end1 = 0x00060005u + seed, begw = 0x00010002u;
    bsw::PkRow r;
    r.glo = 0; r.gsp = 100;
    r.gfa = 0; r.gfn = MODE == 0 ? 100 : 0;
    if (MODE == 2) r.glo = 1000;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
        bsw::pk_group<0>(hh[0], hh[1], hh[2], hh[3], ee[0], ee[1], ee[2], ee[3], hh[4], qp[0], qp[1], hc, hg, f,
                         key, lp, tw, tl, th, end1, begw, 0x00070007u, 0x00010001u, r);
        bsw::pk_group<1>(hh[4], hh[5], hh[6], hh[7], ee[4], ee[5], ee[6], ee[7], hh[8], qp[2], qp[3], hc, hg, f,
                         key, lp, tw, tl, th, end1, begw, 0x00070007u, 0x00010001u, r);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = hc ^ hg ^ f ^ key ^ lp;
#pragma unroll
    for (int k = 0; k < 8; ++k) x ^= hh[k] ^ ee[k];
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = (t1 - t0) + (x == 12345u);
}

template <int MODE> static void run(unsigned long long *d, std::vector<unsigned long long> &h)
{
    const int blocks = 256;
    hipLaunchKernelGGL(kgrp<MODE>, dim3(blocks), dim3(256), 0, 0, d, 1);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(kgrp<MODE>, dim3(blocks), dim3(256), 0, 0, d, 2);
    (void)hipDeviceSynchronize();
    const int nw = blocks * 4;
    (void)hipMemcpy(h.data(), d, nw * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.begin() + nw);
    static const char *names[] = {"fast", "masked", "skip"};
    printf("pk_group %-7s  cycles/group (one wave per SIMD) = %7.1f\n", names[MODE], (double)h[nw / 2] / (2.0 * ITERS));
}
int main()
{
    unsigned long long *d; (void)hipMalloc(&d, 256 * 4 * 8);
    std::vector<unsigned long long> h(256 * 4);
    run<0>(d, h); run<1>(d, h); run<2>(d, h);
    return 0;
}
