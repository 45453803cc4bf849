// Issue-cost microbenchmark for the instruction forms used by the banded-SW cell
// (tools only; not part of the product).  For each pattern a wave runs ITERS x 16
// instructions; s_memtime brackets the loop; cycles/instruction per wave is reported as the
// median over waves, for 1..4 waves per SIMD (grid = 256 CUs x k blocks of 4 waves).
//
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/valu_issue_bench tools/valu_issue_bench.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define ITERS 4096

#define R16(x) x x x x x x x x x x x x x x x x

template <int P>
__global__ __launch_bounds__(256) void kern(unsigned long long* out, int seed) {
  unsigned a = threadIdx.x + seed, b = a * 3u + 1, c = a ^ 0x5555, d = a + 7, e = a * 5u, f = a + 11,
           g = a * 13u, h = a + 17;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (P == 0) {  // independent v_max_i32 (8 regs round robin)
      asm volatile(R16("v_max_i32 %0, %0, %8\n v_max_i32 %1, %1, %8\n v_max_i32 %2, %2, %8\n v_max_i32 %3, %3, %8\n"
                       "v_max_i32 %4, %4, %8\n v_max_i32 %5, %5, %8\n v_max_i32 %6, %6, %8\n v_max_i32 %7, %7, %8\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(seed));
    } else if constexpr (P == 1) {  // dependent chain v_max_i32
      asm volatile(R16("v_max_i32 %0, %0, %1\n v_max_i32 %0, %0, %2\n v_max_i32 %0, %0, %1\n v_max_i32 %0, %0, %2\n"
                       "v_max_i32 %0, %0, %1\n v_max_i32 %0, %0, %2\n v_max_i32 %0, %0, %1\n v_max_i32 %0, %0, %2\n")
                   : "+v"(a) : "v"(b), "v"(c));
    } else if constexpr (P == 2) {  // dependent chain v_max3_i32 (VOP3)
      asm volatile(R16("v_max3_i32 %0, %0, %1, 0\n v_max3_i32 %0, %0, %2, 0\n v_max3_i32 %0, %0, %1, 0\n v_max3_i32 %0, %0, %2, 0\n"
                       "v_max3_i32 %0, %0, %1, 0\n v_max3_i32 %0, %0, %2, 0\n v_max3_i32 %0, %0, %1, 0\n v_max3_i32 %0, %0, %2, 0\n")
                   : "+v"(a) : "v"(b), "v"(c));
    } else if constexpr (P == 3) {  // independent SDWA (word select)
      asm volatile(R16("v_max_i32_sdwa %0, %0, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %1, %1, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %2, %2, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %3, %3, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %4, %4, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %5, %5, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %6, %6, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %7, %7, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(seed));
    } else if constexpr (P == 4) {  // dependent chain SDWA
      asm volatile(R16("v_max_i32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %0, %0, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n"
                       "v_max_i32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %0, %0, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n"
                       "v_max_i32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %0, %0, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n"
                       "v_max_i32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
                       "v_max_i32_sdwa %0, %0, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n")
                   : "+v"(a) : "v"(b), "v"(c));
    } else if constexpr (P == 5) {  // independent v_perm_b32
      asm volatile(R16("v_perm_b32 %0, %8, %9, %0\n v_perm_b32 %1, %8, %9, %1\n v_perm_b32 %2, %8, %9, %2\n v_perm_b32 %3, %8, %9, %3\n"
                       "v_perm_b32 %4, %8, %9, %4\n v_perm_b32 %5, %8, %9, %5\n v_perm_b32 %6, %8, %9, %6\n v_perm_b32 %7, %8, %9, %7\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(seed), "v"(seed + 1));
    } else if constexpr (P == 6) {  // independent v_pk_max_i16
      asm volatile(R16("v_pk_max_i16 %0, %0, %8\n v_pk_max_i16 %1, %1, %8\n v_pk_max_i16 %2, %2, %8\n v_pk_max_i16 %3, %3, %8\n"
                       "v_pk_max_i16 %4, %4, %8\n v_pk_max_i16 %5, %5, %8\n v_pk_max_i16 %6, %6, %8\n v_pk_max_i16 %7, %7, %8\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(seed));
    } else if constexpr (P == 7) {  // dependent v_pk_max_i16 chain
      asm volatile(R16("v_pk_max_i16 %0, %0, %1\n v_pk_max_i16 %0, %0, %2\n v_pk_max_i16 %0, %0, %1\n v_pk_max_i16 %0, %0, %2\n"
                       "v_pk_max_i16 %0, %0, %1\n v_pk_max_i16 %0, %0, %2\n v_pk_max_i16 %0, %0, %1\n v_pk_max_i16 %0, %0, %2\n")
                   : "+v"(a) : "v"(b), "v"(c));
    } else if constexpr (P == 8) {  // two chains interleaved (dependency distance 2)
      asm volatile(R16("v_max_i32 %0, %0, %2\n v_max_i32 %1, %1, %2\n v_max_i32 %0, %0, %2\n v_max_i32 %1, %1, %2\n"
                       "v_max_i32 %0, %0, %2\n v_max_i32 %1, %1, %2\n v_max_i32 %0, %0, %2\n v_max_i32 %1, %1, %2\n")
                   : "+v"(a), "+v"(b) : "v"(seed));
    } else if constexpr (P == 9) {  // independent VALU with one SALU per 4 VALU (SALU counted as instr)
      asm volatile(R16("v_max_i32 %0, %0, %8\n v_max_i32 %1, %1, %8\n v_max_i32 %2, %2, %8\n v_max_i32 %3, %3, %8\n s_add_u32 s10, s10, 1\n"
                       "v_max_i32 %4, %4, %8\n v_max_i32 %5, %5, %8\n v_max_i32 %6, %6, %8\n v_max_i32 %7, %7, %8\n s_add_u32 s11, s11, 1\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(seed) : "s10", "s11", "scc");
    } else if constexpr (P == 10) {  // independent v_cndmask with vcc
      asm volatile("v_cmp_gt_i32 vcc, %0, %1\n" R16("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n"
                       "v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(seed) : "vcc");
    } else if constexpr (P == 11) {  // independent VOP3 v_max3_i32
      asm volatile(R16("v_max3_i32 %0, %0, %8, 0\n v_max3_i32 %1, %1, %8, 0\n v_max3_i32 %2, %2, %8, 0\n v_max3_i32 %3, %3, %8, 0\n"
                       "v_max3_i32 %4, %4, %8, 0\n v_max3_i32 %5, %5, %8, 0\n v_max3_i32 %6, %6, %8, 0\n v_max3_i32 %7, %7, %8, 0\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(seed));
    } else if constexpr (P == 12) {  // dependent 16-bit VOP3 with op_sel (v_max3_i16 hi-half read)
      asm volatile(R16("v_max3_i16 %0, %0, %1, 0 op_sel:[0,1,0,0]\n v_max3_i16 %0, %0, %2, 0 op_sel:[0,1,0,0]\n"
                       "v_max3_i16 %0, %0, %1, 0 op_sel:[0,1,0,0]\n v_max3_i16 %0, %0, %2, 0 op_sel:[0,1,0,0]\n"
                       "v_max3_i16 %0, %0, %1, 0 op_sel:[0,1,0,0]\n v_max3_i16 %0, %0, %2, 0 op_sel:[0,1,0,0]\n"
                       "v_max3_i16 %0, %0, %1, 0 op_sel:[0,1,0,0]\n v_max3_i16 %0, %0, %2, 0 op_sel:[0,1,0,0]\n")
                   : "+v"(a) : "v"(b), "v"(c));
    } else if constexpr (P == 13) {  // realistic cell mix: 4 independent cells' phase-1 (SDWA) then serial F chain
      asm volatile(R16("v_sub_u32_sdwa %0, %4, %5 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n"
                       "v_min_i32_sdwa %1, sext(%6), %4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:WORD_0\n"
                       "v_subrev_u32 %2, %5, %2\n"
                       "v_max3_i32 %2, %2, %1, 0\n"
                       "v_max_i32 %3, %1, %2\n"
                       "v_lshl_or_b32 %4, %0, 16, %3\n"
                       "v_subrev_u32 %2, %5, %2\n"
                       "v_max3_i32 %2, %2, %0, 0\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e) : "v"(f), "v"(g));
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0)
    out[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = (t1 - t0) + ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h) == 12345u ? 1 : 0);
}

static const char* kNames[] = {"indep v_max_i32",  "dep   v_max_i32",     "dep   v_max3_i32 (VOP3)",
                               "indep v_max_i32_sdwa", "dep   v_max_i32_sdwa", "indep v_perm_b32",
                               "indep v_pk_max_i16",   "dep   v_pk_max_i16",   "2 chains interleaved",
                               "indep VALU + 1 SALU/4", "indep v_cndmask vcc",  "indep v_max3_i32",
                               "dep   v_max3_i16 op_sel", "cell mix (8 instr)"};
static const int kInstrPer16[] = {128, 128, 128, 128, 128, 128, 128, 128, 128, 160, 128, 128, 128, 128};

template <int P>
static void run(int k, unsigned long long* d, std::vector<unsigned long long>& h) {
  int blocks = 256 * k;
  hipLaunchKernelGGL(kern<P>, dim3(blocks), dim3(256), 0, 0, d, 1);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern<P>, dim3(blocks), dim3(256), 0, 0, d, 2);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  int nw = blocks * 4;
  hipMemcpy(h.data(), d, nw * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.begin() + nw);
  double med = (double)h[nw / 2];
  double ninstr = (double)ITERS * kInstrPer16[P];
  // chip VALU rate: wave-instructions per SIMD per cycle from wall time needs the clock; report
  // per-wave cycles/instr (s_memtime ticks) and the implied SIMD issue interval (÷ waves/SIMD).
  printf("%-26s waves/SIMD=%d  cyc/instr/wave=%6.2f  SIMD interval=%5.2f  wall=%.3f ms\n", kNames[P], k,
         med / ninstr, med / ninstr / k, ms);
}

template <int P>
static void runall(unsigned long long* d, std::vector<unsigned long long>& h) {
  for (int k = 1; k <= 4; ++k) run<P>(k, d, h);
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 256 * 4 * 4 * 8);
  std::vector<unsigned long long> h(256 * 4 * 4);
  runall<0>(d, h); runall<1>(d, h); runall<2>(d, h); runall<3>(d, h); runall<4>(d, h);
  runall<5>(d, h); runall<6>(d, h); runall<7>(d, h); runall<8>(d, h); runall<9>(d, h);
  runall<10>(d, h); runall<11>(d, h); runall<12>(d, h); runall<13>(d, h);
  hipFree(d);
  return 0;
}
