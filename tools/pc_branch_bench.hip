// Branch-structure cost of the packed-column kernel's FAST group (tools only): the same 34-VALU
// FAST body (bsw_pc.hip) run 8 groups x ITERS per wave with
//   V0: no scalar tests            V1: 2 not-taken test+branch pairs (skip / fast tests)
//   V2: V1 + the taken s_branch over the masked bodies (the product layout)
//   V3: V1 + a taken branch every 2nd group
//   V4: V0 + the 6 byte-unpack/repack v_perm of a narrow (8-bit stored H and E) row, the C3
//       "int8 cells" variant: 4 columns per VGPR for H and E halves the row's registers (3-4
//       waves per SIMD instead of 2) but adds these instructions to every group
// at 1, 2 and 3 waves per SIMD (grid = 1024 * k one-wave blocks).
// build: hipcc -O3 --offload-arch=gfx950 -o tools/pc_branch_bench tools/pc_branch_bench.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
#define ITERS 512

#define PC_SDWA(op, d, a, b, sel) \
    op "_sdwa " d ", " a ", " b " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" sel "\n\t"
#define PC_PH1(X, EOUT)                                                                 \
    "v_pk_min_i16 %[s" X "], %[s" X "], %[h" X "]\n\t"                                      \
    "v_pk_add_u16 %[s" X "], %[s" X "], %[h" X "]\n\t"                                      \
    "v_pk_sub_i16 %[t" X "], %[s" X "], %[oe2]\n\t"                                         \
    "v_pk_max_i16 %[s" X "], %[s" X "], %[e" X "]\n\t"                                      \
    "v_pk_sub_i16 " EOUT ", %[e" X "], %[ed2]\n\t"                                          \
    "v_pk_max_i16 " EOUT ", " EOUT ", %[t" X "]\n\t"
#define PC_SCORES                                                                        \
    "v_perm_b32 %[y], %[phi], %[plo], %[q]\n\t"                                              \
    "v_pk_lshlrev_b16 %[sa], 8, %[y] op_sel_hi:[0,1]\n\t"                                    \
    "v_pk_ashrrev_i16 %[sa], 8, %[sa] op_sel_hi:[0,1]\n\t"                                   \
    "v_pk_ashrrev_i16 %[sb], 8, %[y] op_sel_hi:[0,1]\n\t"
#define PC_CELL(C, X, W)                                                                 \
    PC_SDWA("v_max_i32", C, "%[f]", "sext(%[s" X "])", W)                                    \
    "v_subrev_u32_e64 %[f], %[ed], %[f] clamp\n\t"                                           \
    PC_SDWA("v_max_i32", "%[f]", "%[f]", "sext(%[t" X "])", W)
#define FAST_BODY                                                                        \
        PC_PH1("a", "%[ea]") PC_PH1("b", "%[eb]")                                            \
        PC_CELL("%[c0]", "a", "WORD_0")                                                      \
        PC_CELL("%[c1]", "a", "WORD_1")                                                      \
        "v_lshl_or_b32 %[ha], %[c0], 16, %[h1]\n\t"                                          \
        PC_CELL("%[c2]", "b", "WORD_0")                                                      \
        PC_CELL("%[h1]", "b", "WORD_1")                                                      \
        "v_lshl_or_b32 %[hb], %[c2], 16, %[c1]\n\t"                                          \
        "v_lshl_or_b32 %[pa], %[ha], 8, %[jja]\n\t"                                          \
        "v_pk_max_u16 %[key], %[key], %[pa]\n\t"                                             \
        "v_lshl_or_b32 %[pb], %[hb], 8, %[jjb]\n\t"                                          \
        "v_pk_max_u16 %[key], %[key], %[pb]\n\t"

template <int V>
__device__ __forceinline__ void grp(uint32_t &ha, uint32_t &hb, uint32_t &ea, uint32_t &eb, uint32_t q,
                                    uint32_t plo, uint32_t phi, uint32_t &f, uint32_t &h1, uint32_t &key,
                                    uint64_t men, uint64_t mfa, int G)
{
    uint32_t y, sa, sb, ta, tb, c0, c1, c2, pa, pb;
    if constexpr (V == 4) {
        uint32_t u0, u1;
        asm volatile("v_perm_b32 %[u0], 0, %[ha], %[s0]\n\t"     /* bytes -> int16 pairs */
                     "v_perm_b32 %[u1], 0, %[ha], %[s1]\n\t"
                     "v_perm_b32 %[ea], 0, %[eb], %[s0]\n\t"
                     "v_perm_b32 %[eb], 0, %[eb], %[s1]\n\t"
                     : [u0] "=&v"(u0), [u1] "=&v"(u1), [ea] "+v"(ea), [eb] "+v"(eb)
                     : [ha] "v"(ha), [s0] "s"(0x0c010c00u), [s1] "s"(0x0c030c02u));
        ha = u0; hb = u1;
        asm volatile(PC_SCORES FAST_BODY
            : [ha] "+v"(ha), [hb] "+v"(hb), [ea] "+v"(ea), [eb] "+v"(eb), [f] "+v"(f), [h1] "+v"(h1), [key] "+v"(key),
              [y] "=&v"(y), [sa] "=&v"(sa), [sb] "=&v"(sb), [ta] "=&v"(ta), [tb] "=&v"(tb), [c0] "=&v"(c0),
              [c1] "=&v"(c1), [c2] "=&v"(c2), [pa] "=&v"(pa), [pb] "=&v"(pb)
            : [q] "v"(q), [plo] "v"(plo), [phi] "v"(phi), [oe2] "s"(0x70007u), [ed2] "s"(0x10001u), [ed] "s"(1),
              [jja] "s"(0x40003u), [jjb] "s"(0x60005u));
        asm volatile("v_perm_b32 %[ha], %[hb], %[ha], %[s2]\n\t"   /* int16 pairs -> bytes */
                     "v_perm_b32 %[ea], %[eb], %[ea], %[s2]\n\t"
                     : [ha] "+v"(ha), [ea] "+v"(ea) : [hb] "v"(hb), [eb] "v"(eb), [s2] "s"(0x06040200u));
    } else if constexpr (V == 0) {
        asm volatile(PC_SCORES FAST_BODY
            : [ha] "+v"(ha), [hb] "+v"(hb), [ea] "+v"(ea), [eb] "+v"(eb), [f] "+v"(f), [h1] "+v"(h1), [key] "+v"(key),
              [y] "=&v"(y), [sa] "=&v"(sa), [sb] "=&v"(sb), [ta] "=&v"(ta), [tb] "=&v"(tb), [c0] "=&v"(c0),
              [c1] "=&v"(c1), [c2] "=&v"(c2), [pa] "=&v"(pa), [pb] "=&v"(pb)
            : [q] "v"(q), [plo] "v"(plo), [phi] "v"(phi), [oe2] "s"(0x70007u), [ed2] "s"(0x10001u), [ed] "s"(1),
              [jja] "s"(0x40003u), [jjb] "s"(0x60005u));
    } else if constexpr (V == 1) {
        asm volatile("s_bitcmp1_b64 %[men], %[g]\n\ts_cbranch_scc0 3f\n\t" PC_SCORES
                     "s_bitcmp1_b64 %[mfa], %[g]\n\ts_cbranch_scc0 3f\n\t" FAST_BODY "3:"
            : [ha] "+v"(ha), [hb] "+v"(hb), [ea] "+v"(ea), [eb] "+v"(eb), [f] "+v"(f), [h1] "+v"(h1), [key] "+v"(key),
              [y] "=&v"(y), [sa] "=&v"(sa), [sb] "=&v"(sb), [ta] "=&v"(ta), [tb] "=&v"(tb), [c0] "=&v"(c0),
              [c1] "=&v"(c1), [c2] "=&v"(c2), [pa] "=&v"(pa), [pb] "=&v"(pb)
            : [q] "v"(q), [plo] "v"(plo), [phi] "v"(phi), [oe2] "s"(0x70007u), [ed2] "s"(0x10001u), [ed] "s"(1),
              [jja] "s"(0x40003u), [jjb] "s"(0x60005u), [men] "s"(men), [mfa] "s"(mfa), [g] "s"(G)
            : "scc");
    } else {
        // V2: taken s_branch over a (never run) masked body after every FAST body; V3: every 2nd group
        if (V == 2 || (G & 1))
            asm volatile("s_bitcmp1_b64 %[men], %[g]\n\ts_cbranch_scc0 3f\n\t" PC_SCORES
                         "s_bitcmp1_b64 %[mfa], %[g]\n\ts_cbranch_scc0 2f\n\t" FAST_BODY "s_branch 3f\n"
                         "2:\n\t" FAST_BODY FAST_BODY "3:"
                : [ha] "+v"(ha), [hb] "+v"(hb), [ea] "+v"(ea), [eb] "+v"(eb), [f] "+v"(f), [h1] "+v"(h1), [key] "+v"(key),
                  [y] "=&v"(y), [sa] "=&v"(sa), [sb] "=&v"(sb), [ta] "=&v"(ta), [tb] "=&v"(tb), [c0] "=&v"(c0),
                  [c1] "=&v"(c1), [c2] "=&v"(c2), [pa] "=&v"(pa), [pb] "=&v"(pb)
                : [q] "v"(q), [plo] "v"(plo), [phi] "v"(phi), [oe2] "s"(0x70007u), [ed2] "s"(0x10001u), [ed] "s"(1),
                  [jja] "s"(0x40003u), [jjb] "s"(0x60005u), [men] "s"(men), [mfa] "s"(mfa), [g] "s"(G)
                : "scc");
        else
            asm volatile("s_bitcmp1_b64 %[men], %[g]\n\ts_cbranch_scc0 3f\n\t" PC_SCORES
                         "s_bitcmp1_b64 %[mfa], %[g]\n\ts_cbranch_scc0 3f\n\t" FAST_BODY "3:"
                : [ha] "+v"(ha), [hb] "+v"(hb), [ea] "+v"(ea), [eb] "+v"(eb), [f] "+v"(f), [h1] "+v"(h1), [key] "+v"(key),
                  [y] "=&v"(y), [sa] "=&v"(sa), [sb] "=&v"(sb), [ta] "=&v"(ta), [tb] "=&v"(tb), [c0] "=&v"(c0),
                  [c1] "=&v"(c1), [c2] "=&v"(c2), [pa] "=&v"(pa), [pb] "=&v"(pb)
                : [q] "v"(q), [plo] "v"(plo), [phi] "v"(phi), [oe2] "s"(0x70007u), [ed2] "s"(0x10001u), [ed] "s"(1),
                  [jja] "s"(0x40003u), [jjb] "s"(0x60005u), [men] "s"(men), [mfa] "s"(mfa), [g] "s"(G)
                : "scc");
    }
}

template <int V>
__global__ __launch_bounds__(64) void kern(unsigned long long *out, int seed)
{
    uint32_t hh[16], ee[16];
    for (int k = 0; k < 16; ++k) { hh[k] = (threadIdx.x * 7 + k * 3 + seed) & 0x007f007f; ee[k] = (k * 5) & 0x001f001f; }
    uint32_t q0 = 0x01020304u ^ threadIdx.x, q1 = 0x03000102u, plo = 0xfcfcfc01u, phi = 0xffffffffu;
    uint32_t f = 0, h1 = 3, key = 0;
    const uint64_t men = ~0ull, mfa = ~0ull;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int g = 0; g < 8; ++g)
            grp<V>(hh[2 * g], hh[2 * g + 1], ee[2 * g], ee[2 * g + 1], (g & 1) ? q1 : q0, plo, phi, f, h1, key, men,
                   mfa, g);
        f = 0;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = key ^ h1;
    for (int k = 0; k < 16; ++k) x ^= hh[k] ^ ee[k];
    if ((threadIdx.x & 63) == 0) out[blockIdx.x] = (t1 - t0) + (x == 0x12345678u);
}

static const char *kNames[] = {"V0 no tests", "V1 2 not-taken tests", "V2 + taken branch/group",
                               "V3 + taken branch/2 groups", "V4 V0 + narrow-row unpack/repack"};
template <int V> static void run(int k, unsigned long long *d, std::vector<unsigned long long> &h)
{
    const int blocks = 1024 * k;
    hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(64), 0, 0, d, 1);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(64), 0, 0, d, 2);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(h.data(), d, blocks * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.begin() + blocks);
    const double groups = (double)ITERS * 8;
    printf("%-30s k=%d  wave cyc/group=%7.1f  SIMD cyc/group (wall, 2.4 GHz)=%7.1f\n", kNames[V], k,
           (double)h[blocks / 2] / groups, ms * 1e-3 * 2.4e9 / (k * groups));
}
int main()
{
    unsigned long long *d; (void)hipMalloc(&d, 1024 * 4 * 8);
    std::vector<unsigned long long> h(1024 * 4);
    for (int k = 1; k <= 4; ++k) { run<0>(k, d, h); run<1>(k, d, h); run<2>(k, d, h); run<3>(k, d, h); run<4>(k, d, h); }
    return 0;
}
