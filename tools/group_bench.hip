// Cycle cost of one 4-column group body of the lane kernel (tools only).  OLD = the int16 body in
// bsw_kernels.hip (fast path); NEW/NEWNL = the 16-bit fast-op body with and without lastH tracking.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/group_bench tools/group_bench.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
#define ITERS 1024

#define OLD_BODY \
  "v_perm_b32 %[pw], %[phi], %[plo], %[q]\n" \
  "v_sub_u32_sdwa %[x0], %[v0], %[ed] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
  "v_sub_u32_sdwa %[x1], %[v1], %[ed] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
  "v_sub_u32_sdwa %[x2], %[v2], %[ed] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
  "v_sub_u32_sdwa %[x3], %[v3], %[ed] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n" \
  "v_min_i32_sdwa %[m0], sext(%[pw]), %[v0] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:WORD_0\n" \
  "v_min_i32_sdwa %[m1], sext(%[pw]), %[v1] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:WORD_0\n" \
  "v_min_i32_sdwa %[m2], sext(%[pw]), %[v2] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:WORD_0\n" \
  "v_min_i32_sdwa %[m3], sext(%[pw]), %[v3] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:WORD_0\n" \
  "v_add_u32_sdwa %[m0], %[m0], %[v0] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n" \
  "v_add_u32_sdwa %[m1], %[m1], %[v1] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n" \
  "v_add_u32_sdwa %[m2], %[m2], %[v2] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n" \
  "v_add_u32_sdwa %[m3], %[m3], %[v3] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n" \
  "v_subrev_u32_e32 %[t0], %[oe], %[m0]\n" \
  "v_subrev_u32_e32 %[t1], %[oe], %[m1]\n" \
  "v_subrev_u32_e32 %[t2], %[oe], %[m2]\n" \
  "v_subrev_u32_e32 %[t3], %[oe], %[m3]\n" \
  "v_max_i32_sdwa %[m0], %[m0], %[v0] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n" \
  "v_max_i32_sdwa %[m1], %[m1], %[v1] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n" \
  "v_max_i32_sdwa %[m2], %[m2], %[v2] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n" \
  "v_max_i32_sdwa %[m3], %[m3], %[v3] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n" \
  "v_max3_i32 %[x0], %[x0], %[t0], 0\n" \
  "v_max3_i32 %[x1], %[x1], %[t1], 0\n" \
  "v_max3_i32 %[x2], %[x2], %[t2], 0\n" \
  "v_max3_i32 %[x3], %[x3], %[t3], 0\n" \
  "v_max_i32_e32 %[ha], %[f], %[m0]\n" \
  "v_subrev_u32_e32 %[f], %[ed], %[f]\n" \
  "v_lshl_or_b32 %[v0], %[x0], 16, %[h1]\n" \
  "v_max3_i32 %[f], %[f], %[t0], 0\n" \
  "v_lshlrev_b32_e32 %[m0], 16, %[ha]\n" \
  "v_max_i32_e32 %[hb], %[f], %[m1]\n" \
  "v_subrev_u32_e32 %[f], %[ed], %[f]\n" \
  "v_or_b32_e32 %[k0], 5, %[m0]\n" \
  "v_max3_i32 %[f], %[f], %[t1], 0\n" \
  "v_min_i32_e32 %[l0], 6, %[m0]\n" \
  "v_lshl_or_b32 %[v1], %[x1], 16, %[ha]\n" \
  "v_lshlrev_b32_e32 %[m1], 16, %[hb]\n" \
  "v_max_i32_e32 %[ha], %[f], %[m2]\n" \
  "v_subrev_u32_e32 %[f], %[ed], %[f]\n" \
  "v_or_b32_e32 %[k1], 6, %[m1]\n" \
  "v_max3_i32 %[f], %[f], %[t2], 0\n" \
  "v_min_i32_e32 %[l1], 7, %[m1]\n" \
  "v_lshl_or_b32 %[v2], %[x2], 16, %[hb]\n" \
  "v_max3_i32 %[key], %[key], %[k0], %[k1]\n" \
  "v_lshlrev_b32_e32 %[m2], 16, %[ha]\n" \
  "v_max3_i32 %[lp], %[lp], %[l0], %[l1]\n" \
  "v_max_i32_e32 %[h1], %[f], %[m3]\n" \
  "v_subrev_u32_e32 %[f], %[ed], %[f]\n" \
  "v_or_b32_e32 %[k0], 7, %[m2]\n" \
  "v_max3_i32 %[f], %[f], %[t3], 0\n" \
  "v_min_i32_e32 %[l0], 8, %[m2]\n" \
  "v_lshl_or_b32 %[v3], %[x3], 16, %[ha]\n" \
  "v_lshlrev_b32_e32 %[m3], 16, %[h1]\n" \
  "v_or_b32_e32 %[k1], 8, %[m3]\n" \
  "v_min_i32_e32 %[l1], 9, %[m3]\n" \
  "v_max3_i32 %[key], %[key], %[k0], %[k1]\n" \
  "v_max3_i32 %[lp], %[lp], %[l0], %[l1]\n"

#define NEW_P1 \
  "v_perm_b32 %[pw], %[phi], %[plo], %[q]\n" \
  "v_min_i16_sdwa %[m0], sext(%[pw]), %[v0] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:WORD_0\n" \
  "v_min_i16_sdwa %[m1], sext(%[pw]), %[v1] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:WORD_0\n" \
  "v_min_i16_sdwa %[m2], sext(%[pw]), %[v2] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:WORD_0\n" \
  "v_min_i16_sdwa %[m3], sext(%[pw]), %[v3] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:WORD_0\n" \
  "v_lshrrev_b32 %[x0], 16, %[v0]\n" \
  "v_lshrrev_b32 %[x1], 16, %[v1]\n" \
  "v_lshrrev_b32 %[x2], 16, %[v2]\n" \
  "v_lshrrev_b32 %[x3], 16, %[v3]\n" \
  "v_add_u16 %[m0], %[m0], %[v0]\n" \
  "v_add_u16 %[m1], %[m1], %[v1]\n" \
  "v_add_u16 %[m2], %[m2], %[v2]\n" \
  "v_add_u16 %[m3], %[m3], %[v3]\n" \
  "v_subrev_u16 %[t0], %[oe], %[m0]\n" \
  "v_subrev_u16 %[t1], %[oe], %[m1]\n" \
  "v_subrev_u16 %[t2], %[oe], %[m2]\n" \
  "v_subrev_u16 %[t3], %[oe], %[m3]\n" \
  "v_max_i16 %[m0], %[m0], %[x0]\n" \
  "v_max_i16 %[m1], %[m1], %[x1]\n" \
  "v_max_i16 %[m2], %[m2], %[x2]\n" \
  "v_max_i16 %[m3], %[m3], %[x3]\n" \
  "v_max_i16 %[t0], 0, %[t0]\n" \
  "v_max_i16 %[t1], 0, %[t1]\n" \
  "v_max_i16 %[t2], 0, %[t2]\n" \
  "v_max_i16 %[t3], 0, %[t3]\n" \
  "v_subrev_u16 %[x0], %[ed], %[x0]\n" \
  "v_subrev_u16 %[x1], %[ed], %[x1]\n" \
  "v_subrev_u16 %[x2], %[ed], %[x2]\n" \
  "v_subrev_u16 %[x3], %[ed], %[x3]\n" \
  "v_mov_b32 %[v0], %[h1]\n"

#define NEW_CELL(K, VK, HK, J, J1) \
  "v_max_i16 " HK ", %[m" #K "], %[f]\n" \
  "v_max_i16_sdwa " VK ", %[x" #K "], %[t" #K "] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" \
  "v_subrev_u16 %[f], %[ed], %[f]\n" \
  "v_lshlrev_b16 %[ka], 8, " HK "\n" \
  "v_max_i16 %[f], %[f], %[t" #K "]\n" \
  "v_or_b32 %[ka], " J ", %[ka]\n" \
  "v_max_u16 %[key], %[key], %[ka]\n"
#define NEW_LP(J1) \
  "v_min_u16 %[kb], " J1 ", %[ka]\n" \
  "v_max_u16 %[lp], %[lp], %[kb]\n"

#define NEW_BODY NEW_P1 \
  NEW_CELL(0, "%[v0]", "%[v1]", "5", "6") NEW_LP("0x106") \
  NEW_CELL(1, "%[v1]", "%[v2]", "6", "7") NEW_LP("0x107") \
  NEW_CELL(2, "%[v2]", "%[v3]", "7", "8") NEW_LP("0x108") \
  NEW_CELL(3, "%[v3]", "%[h1]", "8", "9") NEW_LP("0x109")
#define NEWNL_BODY NEW_P1 \
  NEW_CELL(0, "%[v0]", "%[v1]", "5", "6") \
  NEW_CELL(1, "%[v1]", "%[v2]", "6", "7") \
  NEW_CELL(2, "%[v2]", "%[v3]", "7", "8") \
  NEW_CELL(3, "%[v3]", "%[h1]", "8", "9")

template <int P>
__global__ __launch_bounds__(256) void kern(unsigned long long* out, int seed, int oe_, int ed_) {
  uint32_t v0 = threadIdx.x * 3 + seed, v1 = v0 ^ 0x10005, v2 = v0 + 0x20007, v3 = v0 * 5;
  uint32_t q = 0x01020304u ^ threadIdx.x, plo = 0xfcfcfc01u, phi = 0xffffffffu;
  int f = 3, h1 = 7, key = 0, lp = 0;
  int m0, m1, m2, m3, t0, t1, t2, t3, x0, x1, x2, x3, ha, hb, k0, k1, l0, l1, pw, ka, kb;
  unsigned long long t0c = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#define OPS : [v0] "+v"(v0), [v1] "+v"(v1), [v2] "+v"(v2), [v3] "+v"(v3), [f] "+v"(f), [h1] "+v"(h1), \
              [key] "+v"(key), [lp] "+v"(lp), [m0] "=&v"(m0), [m1] "=&v"(m1), [m2] "=&v"(m2), [m3] "=&v"(m3), \
              [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [x0] "=&v"(x0), [x1] "=&v"(x1), \
              [x2] "=&v"(x2), [x3] "=&v"(x3), [ha] "=&v"(ha), [hb] "=&v"(hb), [k0] "=&v"(k0), [k1] "=&v"(k1), \
              [l0] "=&v"(l0), [l1] "=&v"(l1), [pw] "=&v"(pw), [ka] "=&v"(ka), [kb] "=&v"(kb) \
            : [q] "v"(q), [plo] "v"(plo), [phi] "v"(phi), [oe] "s"(oe_), [ed] "s"(ed_)
    if constexpr (P == 0) asm volatile(OLD_BODY OPS);
    if constexpr (P == 1) asm volatile(NEW_BODY OPS);
    if constexpr (P == 2) asm volatile(NEWNL_BODY OPS);
  }
  unsigned long long t1c = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0)
    out[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = (t1c - t0c) + ((v0 ^ v1 ^ v2 ^ v3 ^ key ^ lp ^ f) == 12345u);
}


#define PK_P1(K, QP, DUP, HH, EE) \
  "v_perm_b32 %[c" #K "], " QP ", " QP ", " DUP "\n" \
  "v_xor_b32 %[c" #K "], %[c" #K "], %[trow]\n" \
  "v_perm_b32 %[c" #K "], %[tabhi], %[tablo], %[c" #K "]\n" \
  "v_pk_min_i16 %[m" #K "], %[c" #K "], " HH "\n" \
  "v_pk_add_u16 %[m" #K "], %[m" #K "], " HH "\n" \
  "v_pk_sub_i16 %[t" #K "], %[m" #K "], %[oe2]\n" \
  "v_pk_max_i16 %[t" #K "], %[t" #K "], 0\n" \
  "v_pk_max_i16 %[m" #K "], %[m" #K "], " EE "\n" \
  "v_pk_sub_i16 %[x" #K "], " EE ", %[ed2]\n" \
  "v_pk_max_i16 " EE ", %[x" #K "], %[t" #K "]\n"
#define PK_P2(K, HOUT, JJ) \
  "v_pk_max_i16 " HOUT ", %[m" #K "], %[f]\n" \
  "v_pk_sub_i16 %[f], %[f], %[ed2]\n" \
  "v_pk_max_i16 %[f], %[f], %[t" #K "]\n" \
  "v_pk_lshlrev_b16 %[ka], 8, " HOUT "\n" \
  "v_or_b32 %[ka], " JJ ", %[ka]\n" \
  "v_pk_max_u16 %[key], %[key], %[ka]\n"
#define PK_BODY \
  PK_P1(0, "%[qp0]", "%[dup0]", "%[h0]", "%[e0]") PK_P1(1, "%[qp0]", "%[dup1]", "%[h1r]", "%[e1]") \
  PK_P1(2, "%[qp1]", "%[dup0]", "%[h2]", "%[e2]") PK_P1(3, "%[qp1]", "%[dup1]", "%[h3]", "%[e3]") \
  "v_mov_b32 %[h0], %[hc]\n" \
  PK_P2(0, "%[h1r]", "0x50005") PK_P2(1, "%[h2]", "0x60006") PK_P2(2, "%[h3]", "0x70007") PK_P2(3, "%[hc]", "0x80008")

template <int P>
__global__ __launch_bounds__(256) void kpk(unsigned long long* out, int seed, int oe_, int ed_) {
  uint32_t h0 = threadIdx.x * 3 + seed, h1r = h0 ^ 0x10005, h2 = h0 + 0x20007, h3 = h0 * 5, hc = 7;
  uint32_t e0 = h0 ^ 0x55, e1 = h0 + 9, e2 = h0 * 7, e3 = h0 ^ 0x1234;
  uint32_t qp0 = 0x01020304u ^ threadIdx.x, qp1 = 0x02030001u, trow = 0x0c000c00u ^ seed;
  uint32_t tablo = 0xfcfcfc01u, tabhi = 0xffffffffu;
  uint32_t f = 3, key = 0;
  uint32_t m0, m1, m2, m3, t0, t1, t2, t3, x0, x1, x2, x3, c0, c1, c2, c3, ka;
  unsigned long long t0c = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile(PK_BODY
      : [h0] "+v"(h0), [h1r] "+v"(h1r), [h2] "+v"(h2), [h3] "+v"(h3), [hc] "+v"(hc), [e0] "+v"(e0), [e1] "+v"(e1),
        [e2] "+v"(e2), [e3] "+v"(e3), [f] "+v"(f), [key] "+v"(key), [m0] "=&v"(m0), [m1] "=&v"(m1), [m2] "=&v"(m2),
        [m3] "=&v"(m3), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [x0] "=&v"(x0), [x1] "=&v"(x1),
        [x2] "=&v"(x2), [x3] "=&v"(x3), [c0] "=&v"(c0), [c1] "=&v"(c1), [c2] "=&v"(c2), [c3] "=&v"(c3), [ka] "=&v"(ka)
      : [qp0] "v"(qp0), [qp1] "v"(qp1), [trow] "v"(trow), [tablo] "v"(tablo), [tabhi] "v"(tabhi),
        [dup0] "s"(0x01010000), [dup1] "s"(0x03030202), [oe2] "s"(oe_ * 0x10001), [ed2] "s"(ed_ * 0x10001));
  }
  unsigned long long t1c = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0)
    out[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = (t1c - t0c) + ((h0 ^ h1r ^ e0 ^ key ^ f ^ hc) == 12345u);
}
template <int P> static void runpk(int k, unsigned long long* d, std::vector<unsigned long long>& h) {
  int blocks = 256 * k;
  hipLaunchKernelGGL(kpk<P>, dim3(blocks), dim3(256), 0, 0, d, 1, 7, 1);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kpk<P>, dim3(blocks), dim3(256), 0, 0, d, 2, 7, 1);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  int nw = blocks * 4;
  (void)hipMemcpy(h.data(), d, nw * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.begin() + nw);
  printf("%-40s k=%d  wave cyc/group=%7.1f  SIMD cyc/group(wall@2.4GHz)=%7.1f  (8 cells/group)\n",
         "PK 2-pairs/lane group (4 cols x 2 pairs)", k, (double)h[nw / 2] / ITERS, ms * 1e-3 * 2.4e9 / ((double)k * ITERS));
}

static const char* kNames[] = {"OLD int16 fast group (57 VALU)", "NEW 16-bit fast-op group (+lastH)",
                               "NEW 16-bit fast-op group (no lastH)"};
template <int P> static void run(int k, unsigned long long* d, std::vector<unsigned long long>& h) {
  int blocks = 256 * k;
  hipLaunchKernelGGL(kern<P>, dim3(blocks), dim3(256), 0, 0, d, 1, 7, 1);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern<P>, dim3(blocks), dim3(256), 0, 0, d, 2, 7, 1);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  int nw = blocks * 4;
  (void)hipMemcpy(h.data(), d, nw * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.begin() + nw);
  printf("%-40s k=%d  wave cyc/group=%7.1f  SIMD cyc/group(wall@2.4GHz)=%7.1f\n", kNames[P], k,
         (double)h[nw / 2] / ITERS, ms * 1e-3 * 2.4e9 / ((double)k * ITERS));
}
int main() {
  unsigned long long* d; (void)hipMalloc(&d, 256 * 4 * 4 * 8);
  std::vector<unsigned long long> h(256 * 4 * 4);
  for (int k = 1; k <= 2; ++k) { run<0>(k, d, h); runpk<0>(k, d, h); }
  return 0;
}
