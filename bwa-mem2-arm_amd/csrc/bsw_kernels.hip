// bsw_kernels.hip -- CDNA4 (gfx950) kernels for BWA-MEM2 seed extension (banded SW with
// ksw_extend2 semantics; upstream BandedPairWiseSW::getScores16/8, SURVEY.md §3.2-3.3,
// Appendix A).  Written for MI355X: wave64, SIMD-32, 512-entry VGPR file per SIMD lane.
//
// Lane kernel (the hot path)
//   One LANE owns one SeqPair.  The pair's whole DP row eh[0..QMAX] lives in VGPRs as packed
//   {h: bits 0-15, e: bits 16-31} (one VGPR per query column, fully unrolled, compile-time
//   register indices), the query as byte codes (4 per VGPR).  A wavefront therefore advances
//   64 independent alignments through their target rows in lock-step: no cross-lane traffic
//   in the cell loop, no LDS traffic, no HBM traffic except one target byte per row.
//   Per cell (A.4): M = H(i-1,j-1)+S gated by H(i-1,j-1)!=0, H = max(M,E,F),
//   E' = max(E-e_del, M-oe_del, 0), F' = max(F-e_ins, M-oe_ins, 0), row max with last-index
//   argmax, last positive column.  S comes from a per-row profile (v_perm of the query codes
//   against the target base's 8-byte score row) extracted with SDWA byte selects.
//   Band edges are per lane; columns where every live lane is in band run unmasked,
//   edge columns run under per-lane EXEC masks (stale-column rule A.7 preserved exactly).
//
// Wide kernel (fallback): same recurrence, int32 cells, eh row in HBM
//   scratch laid out [column][pair-slot] so a wavefront's accesses are coalesced.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include <utility>
#include "bsw_kernels.h"
#include "bsw_wave.h"


#ifndef BSW_CELL_FENCE
#define BSW_CELL_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif

namespace bsw {

__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

// ------------------------------------------------------------------ lane kernel
struct LaneRow {          // per-row uniform (SGPR) bounds
    int ulo, uhi;         // min beg / max end over live lanes (columns outside: skipped)
    int fast_lo, fast_hi; // max beg / min end over live lanes (columns inside: unmasked)
    int glo, gsp;         // groups touching [ulo, uhi]: glo <= G <= glo + gsp
    int gfa, gfn;         // groups fully inside [fast_lo, fast_hi): gfa <= G < gfa + gfn
    int gua, gun;         // groups whose band edges are wave-uniform or absent: gua <= G < gua + gun
    int usp;              // fast_hi - fast_lo (the uniform span inside those groups)
};

struct LaneCx {           // per-kernel constants
    int e_del, oe_del, e_ins, oe_ins, maxsc;
};

// One DP cell at compile-time column J (SURVEY.md A.4 cell step; A.5-exact form).
//   SM  : 1 -> max(mat) == 1 (bwa -A1): gate M = hold + min(s, hold);  2 -> general max(mat)
//   SYM : o_del == o_ins && e_del == e_ins (bwa default) -> M - oe shared by E and F
// key = max over in-band cells of (H << 16 | j)      -> row max m, ties to the last j
// lp1 = max over in-band cells of min(H << 16, j+1)  -> 1 + last j with H > 0 (0: none)
template <int J, int SM, bool SYM, int NE>
__device__ __forceinline__ void lane_cell(uint32_t (&eh)[NE], int s, int &f, int &h1, int &key,
                                          int &lp1, const LaneCx &c)
{
    const uint32_t v = eh[J];          // { H(i-1,j-1), E(i,j) }
    const int hold = (int)(v & 0xffffu);
    const int e = (int)(v >> 16);
    int M;                              // <= 0 whenever hold == 0 (gate), exact otherwise
    if constexpr (SM == 1) M = hold + min(s, hold);
    else M = hold + min(s, hold * c.maxsc);
    const int h = max3i(M, e, f);       // H(i,j) >= 0, exact
    const int hs = h << 16;
    key = max(key, hs | J);
    lp1 = max(lp1, min(hs, J + 1));
    int e2;
    if constexpr (SYM) {
        const int t = M - c.oe_del;
        e2 = max3i(e - c.e_del, t, 0);  // E(i+1,j)
        f = max3i(f - c.e_del, t, 0);   // F(i,j+1)
    } else {
        e2 = max3i(e - c.e_del, M - c.oe_del, 0);
        f = max3i(f - c.e_ins, M - c.oe_ins, 0);
    }
    eh[J] = (uint32_t)h1 | ((uint32_t)e2 << 16);               // { H(i,j-1), E(i+1,j) }
    h1 = h;
}

// Row structure.  The row's columns are visited as 4-column groups in a
// straight unrolled sequence.  Per group one uniform (SGPR) test decides:
//   skip   : group outside [min beg, max end] of the live lanes;
//   fast   : every live lane is in band for all four columns -> one inline-asm block,
//            no lane masks, eh[]/f/h1/key/lp1 updated IN PLACE (tied "+v" operands);
//   masked : otherwise each column runs under its per-lane EXEC mask (band edges).
// Only the masked path (a few columns per row) pays merge copies.

// Masked column J: per-lane band membership under EXEC; at j == end write
// { H(i,end-1), 0 } (A.4 end of row); beyond end leave eh untouched (A.7 stale columns).
template <int J, int QMAX, int SM, bool SYM>
__device__ __forceinline__ void lane_col_masked(uint32_t (&eh)[QMAX + 1], int s, int beg, int end,
                                                int &f, int &h1, int &key, int &lp1,
                                                const LaneRow &r, const LaneCx &c)
{
    if (J < r.ulo || J > r.uhi) return;                   // uniform
    if constexpr (J < QMAX) {
        if (J >= beg && J < end) {
            lane_cell<J, SM, SYM, QMAX + 1>(eh, s, f, h1, key, lp1, c);
            return;
        }
    }
    if (J == end) eh[J] = (uint32_t)h1;
}

// One 4-column group, default scoring (max(mat) == 1, symmetric gaps), as ONE asm
// statement, so the compiler sees a single in-place update of eh[4G..4G+3], f, h1, key,
// lp1 (no control-flow merge of the DP row, hence no register copies):
//   skip    : group outside [min beg, max end] of the live lanes (scalar test);
//   phase 1 : the four cells' independent work -- M (gated), E' = max(E-e, M-oe, 0),
//             max(M, E), M - oe -- shared by both bodies;
//   fast    : every live lane in band (scalar test): the F chain (2 dependent ops per
//             cell) with H / pack / key interleaved -- 46 VALU per 4 cells (the last positive
//             column is not tracked per cell: lane_lastpos recovers it at row end when needed);
//   masked  : band edges by per-lane SELECTS (no EXEC changes): d = j - beg, in = d < span,
//             inat = d <= span (j == end stores {H(i,end-1), 0}: E' forced to 0), j < beg
//             resets F; out-of-band lanes pass H(i,j-1) along the chain but feed 0 to
//             key -- 82 VALU.
// key = H << 16 | j by one v_lshl_or_b32 with j from an SGPR (VOP3 takes no literal on gfx9).
template <int G>
__device__ __forceinline__ void lane_group_asm(uint32_t &v0, uint32_t &v1, uint32_t &v2, uint32_t &v3,
                                               uint32_t q, uint32_t plo, uint32_t phi, int &f,
                                               int &h1, int &key, int oe, int ed,
                                               int glo, int gsp, int gfa, int gfn, int gua, int gun,
                                               int bs, int usp, int beg, int span)
{
    int m0, m1, m2, m3, t0, t1, t2, t3, x0, x1, x2, x3, ha, hb, k0, k1, pw, st, d, tp;
    uint64_t sat, slt, inb;
    asm volatile(
        "s_sub_u32 %[st], %[g], %[glo]\n\t"     // group outside [min beg, max end]: skip
        "s_cmp_le_u32 %[st], %[gsp]\n\t"
        "s_cbranch_scc0 3f\n\t"
        "v_perm_b32 %[pw], %[phi], %[plo], %[q]\n\t"
        "v_sub_u32_sdwa %[x0], %[v0], %[ed] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
        "v_sub_u32_sdwa %[x1], %[v1], %[ed] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
        "v_sub_u32_sdwa %[x2], %[v2], %[ed] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
        "v_sub_u32_sdwa %[x3], %[v3], %[ed] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
        "v_min_i32_sdwa %[m0], sext(%[pw]), %[v0] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:WORD_0\n\t"
        "v_min_i32_sdwa %[m1], sext(%[pw]), %[v1] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:WORD_0\n\t"
        "v_min_i32_sdwa %[m2], sext(%[pw]), %[v2] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:WORD_0\n\t"
        "v_min_i32_sdwa %[m3], sext(%[pw]), %[v3] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %[m0], %[m0], %[v0] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %[m1], %[m1], %[v1] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %[m2], %[m2], %[v2] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_add_u32_sdwa %[m3], %[m3], %[v3] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_subrev_u32_e32 %[t0], %[oe], %[m0]\n\t"
        "v_subrev_u32_e32 %[t1], %[oe], %[m1]\n\t"
        "v_subrev_u32_e32 %[t2], %[oe], %[m2]\n\t"
        "v_subrev_u32_e32 %[t3], %[oe], %[m3]\n\t"
        "v_max_i32_sdwa %[m0], %[m0], %[v0] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_max_i32_sdwa %[m1], %[m1], %[v1] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_max_i32_sdwa %[m2], %[m2], %[v2] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_max_i32_sdwa %[m3], %[m3], %[v3] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_max3_i32 %[x0], %[x0], %[t0], 0\n\t"
        "v_max3_i32 %[x1], %[x1], %[t1], 0\n\t"
        "v_max3_i32 %[x2], %[x2], %[t2], 0\n\t"
        "v_max3_i32 %[x3], %[x3], %[t3], 0\n\t"
        "s_sub_u32 %[st], %[g], %[gfa]\n\t"     // gfa <= G < gfa + gfn: all lanes in band
        "s_cmp_lt_u32 %[st], %[gfn]\n\t"
        "s_cbranch_scc0 2f\n\t"
        "v_max_i32_e32 %[ha], %[f], %[m0]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_lshl_or_b32 %[v0], %[x0], 16, %[h1]\n\t"
        "v_max3_i32 %[f], %[f], %[t0], 0\n\t"
        "v_lshl_or_b32 %[k0], %[ha], 16, %[s0]\n\t"
        "v_max_i32_e32 %[hb], %[f], %[m1]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_lshl_or_b32 %[v1], %[x1], 16, %[ha]\n\t"
        "v_max3_i32 %[f], %[f], %[t1], 0\n\t"
        "v_lshl_or_b32 %[k1], %[hb], 16, %[s1]\n\t"
        "v_max_i32_e32 %[ha], %[f], %[m2]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_lshl_or_b32 %[v2], %[x2], 16, %[hb]\n\t"
        "v_max3_i32 %[key], %[key], %[k0], %[k1]\n\t"
        "v_max3_i32 %[f], %[f], %[t2], 0\n\t"
        "v_lshl_or_b32 %[k0], %[ha], 16, %[s2]\n\t"
        "v_max_i32_e32 %[h1], %[f], %[m3]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_lshl_or_b32 %[v3], %[x3], 16, %[ha]\n\t"
        "v_max3_i32 %[f], %[f], %[t3], 0\n\t"
        "v_lshl_or_b32 %[k1], %[h1], 16, %[s3]\n\t"
        "v_max3_i32 %[key], %[key], %[k0], %[k1]\n\t"
        "s_branch 3f\n"
        "2:\n\t"
        "s_sub_u32 %[st], %[g], %[gua]\n\t"   // both edges wave-uniform (or absent): U body
        "s_cmp_lt_u32 %[st], %[gun]\n\t"
        "s_cbranch_scc1 5f\n\t"
        "s_cmp_ge_u32 %[g], %[gfa]\n\t"       // no cell left of any lane's beg: R body
        "s_cbranch_scc1 6f\n\t"
        "v_sub_u32_e32 %[d], %[j0], %[beg]\n\t"
        "v_cmp_lt_u32_e64 %[inb], %[d], %[span]\n\t"
        "v_cmp_le_u32_e64 %[sat], %[d], %[span]\n\t"
        "v_cmp_gt_i32_e64 %[slt], 0, %[d]\n\t"
        "v_max_i32_e32 %[tp], %[f], %[m0]\n\t"
        "v_cndmask_b32_e64 %[ha], %[h1], %[tp], %[inb]\n\t"
        "v_cndmask_b32_e64 %[tp], 0, %[tp], %[inb]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_cndmask_b32_e64 %[x0], 0, %[x0], %[inb]\n\t"
        "v_max3_i32 %[f], %[f], %[t0], 0\n\t"
        "v_lshl_or_b32 %[d], %[x0], 16, %[h1]\n\t"
        "v_cndmask_b32_e64 %[f], %[f], 0, %[slt]\n\t"
        "v_cndmask_b32_e64 %[v0], %[v0], %[d], %[sat]\n\t"
        "v_lshl_or_b32 %[k0], %[tp], 16, %[s0]\n\t"
        "v_sub_u32_e32 %[d], %[j1], %[beg]\n\t"
        "v_cmp_lt_u32_e64 %[inb], %[d], %[span]\n\t"
        "v_cmp_le_u32_e64 %[sat], %[d], %[span]\n\t"
        "v_cmp_gt_i32_e64 %[slt], 0, %[d]\n\t"
        "v_max_i32_e32 %[tp], %[f], %[m1]\n\t"
        "v_cndmask_b32_e64 %[hb], %[ha], %[tp], %[inb]\n\t"
        "v_cndmask_b32_e64 %[tp], 0, %[tp], %[inb]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_cndmask_b32_e64 %[x1], 0, %[x1], %[inb]\n\t"
        "v_max3_i32 %[f], %[f], %[t1], 0\n\t"
        "v_lshl_or_b32 %[d], %[x1], 16, %[ha]\n\t"
        "v_cndmask_b32_e64 %[f], %[f], 0, %[slt]\n\t"
        "v_cndmask_b32_e64 %[v1], %[v1], %[d], %[sat]\n\t"
        "v_lshl_or_b32 %[k1], %[tp], 16, %[s1]\n\t"
        "v_max3_i32 %[key], %[key], %[k0], %[k1]\n\t"
        "v_sub_u32_e32 %[d], %[j2], %[beg]\n\t"
        "v_cmp_lt_u32_e64 %[inb], %[d], %[span]\n\t"
        "v_cmp_le_u32_e64 %[sat], %[d], %[span]\n\t"
        "v_cmp_gt_i32_e64 %[slt], 0, %[d]\n\t"
        "v_max_i32_e32 %[tp], %[f], %[m2]\n\t"
        "v_cndmask_b32_e64 %[ha], %[hb], %[tp], %[inb]\n\t"
        "v_cndmask_b32_e64 %[tp], 0, %[tp], %[inb]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_cndmask_b32_e64 %[x2], 0, %[x2], %[inb]\n\t"
        "v_max3_i32 %[f], %[f], %[t2], 0\n\t"
        "v_lshl_or_b32 %[d], %[x2], 16, %[hb]\n\t"
        "v_cndmask_b32_e64 %[f], %[f], 0, %[slt]\n\t"
        "v_cndmask_b32_e64 %[v2], %[v2], %[d], %[sat]\n\t"
        "v_lshl_or_b32 %[k0], %[tp], 16, %[s2]\n\t"
        "v_sub_u32_e32 %[d], %[j3], %[beg]\n\t"
        "v_cmp_lt_u32_e64 %[inb], %[d], %[span]\n\t"
        "v_cmp_le_u32_e64 %[sat], %[d], %[span]\n\t"
        "v_cmp_gt_i32_e64 %[slt], 0, %[d]\n\t"
        "v_max_i32_e32 %[tp], %[f], %[m3]\n\t"
        "v_cndmask_b32_e64 %[h1], %[ha], %[tp], %[inb]\n\t"
        "v_cndmask_b32_e64 %[tp], 0, %[tp], %[inb]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_cndmask_b32_e64 %[x3], 0, %[x3], %[inb]\n\t"
        "v_max3_i32 %[f], %[f], %[t3], 0\n\t"
        "v_lshl_or_b32 %[d], %[x3], 16, %[ha]\n\t"
        "v_cndmask_b32_e64 %[f], %[f], 0, %[slt]\n\t"
        "v_cndmask_b32_e64 %[v3], %[v3], %[d], %[sat]\n\t"
        "v_lshl_or_b32 %[k1], %[tp], 16, %[s3]\n\t"
        "v_max3_i32 %[key], %[key], %[k0], %[k1]\n\t"
        "s_branch 3f\n"
        "5:\n\t"
        "s_sub_u32 %[st], %[j0], %[bs]\n\t"
        "s_cmp_lt_u32 %[st], %[usp]\n\t"
        "s_cbranch_scc0 110f\n\t"
        "v_lshl_or_b32 %[v0], %[x0], 16, %[h1]\n\t"
        "v_max_i32_e32 %[h1], %[f], %[m0]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_max3_i32 %[f], %[f], %[t0], 0\n\t"
        "v_lshl_or_b32 %[k0], %[h1], 16, %[s0]\n\t"
        "v_max_i32_e32 %[key], %[key], %[k0]\n"
        "100:\n\t"
        "s_sub_u32 %[st], %[j1], %[bs]\n\t"
        "s_cmp_lt_u32 %[st], %[usp]\n\t"
        "s_cbranch_scc0 111f\n\t"
        "v_lshl_or_b32 %[v1], %[x1], 16, %[h1]\n\t"
        "v_max_i32_e32 %[h1], %[f], %[m1]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_max3_i32 %[f], %[f], %[t1], 0\n\t"
        "v_lshl_or_b32 %[k0], %[h1], 16, %[s1]\n\t"
        "v_max_i32_e32 %[key], %[key], %[k0]\n"
        "101:\n\t"
        "s_sub_u32 %[st], %[j2], %[bs]\n\t"
        "s_cmp_lt_u32 %[st], %[usp]\n\t"
        "s_cbranch_scc0 112f\n\t"
        "v_lshl_or_b32 %[v2], %[x2], 16, %[h1]\n\t"
        "v_max_i32_e32 %[h1], %[f], %[m2]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_max3_i32 %[f], %[f], %[t2], 0\n\t"
        "v_lshl_or_b32 %[k0], %[h1], 16, %[s2]\n\t"
        "v_max_i32_e32 %[key], %[key], %[k0]\n"
        "102:\n\t"
        "s_sub_u32 %[st], %[j3], %[bs]\n\t"
        "s_cmp_lt_u32 %[st], %[usp]\n\t"
        "s_cbranch_scc0 113f\n\t"
        "v_lshl_or_b32 %[v3], %[x3], 16, %[h1]\n\t"
        "v_max_i32_e32 %[h1], %[f], %[m3]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_max3_i32 %[f], %[f], %[t3], 0\n\t"
        "v_lshl_or_b32 %[k0], %[h1], 16, %[s3]\n\t"
        "v_max_i32_e32 %[key], %[key], %[k0]\n"
        "103:\n\t"
        "s_branch 3f\n"
        "110:\n\t"                          // cell 0 outside the uniform band
        "s_cmp_eq_u32 %[st], %[usp]\n\t"       // j == end: {H(i,end-1), 0}
        "s_cbranch_scc0 100b\n\t"
        "v_mov_b32_e32 %[v0], %[h1]\n\t"
        "s_branch 100b\n"
        "111:\n\t"                          // cell 1 outside the uniform band
        "s_cmp_eq_u32 %[st], %[usp]\n\t"       // j == end: {H(i,end-1), 0}
        "s_cbranch_scc0 101b\n\t"
        "v_mov_b32_e32 %[v1], %[h1]\n\t"
        "s_branch 101b\n"
        "112:\n\t"                          // cell 2 outside the uniform band
        "s_cmp_eq_u32 %[st], %[usp]\n\t"       // j == end: {H(i,end-1), 0}
        "s_cbranch_scc0 102b\n\t"
        "v_mov_b32_e32 %[v2], %[h1]\n\t"
        "s_branch 102b\n"
        "113:\n\t"                          // cell 3 outside the uniform band
        "s_cmp_eq_u32 %[st], %[usp]\n\t"       // j == end: {H(i,end-1), 0}
        "s_cbranch_scc0 103b\n\t"
        "v_mov_b32_e32 %[v3], %[h1]\n\t"
        "s_branch 103b\n"
        "6:\n\t"
        "v_cmp_lt_i32_e64 %[inb], %[s0], %[endv]\n\t"
        "v_cmp_le_i32_e64 %[sat], %[s0], %[endv]\n\t"
        "v_max_i32_e32 %[tp], %[f], %[m0]\n\t"
        "v_cndmask_b32_e64 %[ha], %[h1], %[tp], %[inb]\n\t"
        "v_cndmask_b32_e64 %[tp], 0, %[tp], %[inb]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_cndmask_b32_e64 %[x0], 0, %[x0], %[inb]\n\t"
        "v_max3_i32 %[f], %[f], %[t0], 0\n\t"
        "v_lshl_or_b32 %[d], %[x0], 16, %[h1]\n\t"
        "v_cndmask_b32_e64 %[v0], %[v0], %[d], %[sat]\n\t"
        "v_lshl_or_b32 %[k0], %[tp], 16, %[s0]\n\t"
        "v_cmp_lt_i32_e64 %[inb], %[s1], %[endv]\n\t"
        "v_cmp_le_i32_e64 %[sat], %[s1], %[endv]\n\t"
        "v_max_i32_e32 %[tp], %[f], %[m1]\n\t"
        "v_cndmask_b32_e64 %[hb], %[ha], %[tp], %[inb]\n\t"
        "v_cndmask_b32_e64 %[tp], 0, %[tp], %[inb]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_cndmask_b32_e64 %[x1], 0, %[x1], %[inb]\n\t"
        "v_max3_i32 %[f], %[f], %[t1], 0\n\t"
        "v_lshl_or_b32 %[d], %[x1], 16, %[ha]\n\t"
        "v_cndmask_b32_e64 %[v1], %[v1], %[d], %[sat]\n\t"
        "v_lshl_or_b32 %[k1], %[tp], 16, %[s1]\n\t"
        "v_max3_i32 %[key], %[key], %[k0], %[k1]\n\t"
        "v_cmp_lt_i32_e64 %[inb], %[s2], %[endv]\n\t"
        "v_cmp_le_i32_e64 %[sat], %[s2], %[endv]\n\t"
        "v_max_i32_e32 %[tp], %[f], %[m2]\n\t"
        "v_cndmask_b32_e64 %[ha], %[hb], %[tp], %[inb]\n\t"
        "v_cndmask_b32_e64 %[tp], 0, %[tp], %[inb]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_cndmask_b32_e64 %[x2], 0, %[x2], %[inb]\n\t"
        "v_max3_i32 %[f], %[f], %[t2], 0\n\t"
        "v_lshl_or_b32 %[d], %[x2], 16, %[hb]\n\t"
        "v_cndmask_b32_e64 %[v2], %[v2], %[d], %[sat]\n\t"
        "v_lshl_or_b32 %[k0], %[tp], 16, %[s2]\n\t"
        "v_cmp_lt_i32_e64 %[inb], %[s3], %[endv]\n\t"
        "v_cmp_le_i32_e64 %[sat], %[s3], %[endv]\n\t"
        "v_max_i32_e32 %[tp], %[f], %[m3]\n\t"
        "v_cndmask_b32_e64 %[h1], %[ha], %[tp], %[inb]\n\t"
        "v_cndmask_b32_e64 %[tp], 0, %[tp], %[inb]\n\t"
        "v_subrev_u32_e32 %[f], %[ed], %[f]\n\t"
        "v_cndmask_b32_e64 %[x3], 0, %[x3], %[inb]\n\t"
        "v_max3_i32 %[f], %[f], %[t3], 0\n\t"
        "v_lshl_or_b32 %[d], %[x3], 16, %[ha]\n\t"
        "v_cndmask_b32_e64 %[v3], %[v3], %[d], %[sat]\n\t"
        "v_lshl_or_b32 %[k1], %[tp], 16, %[s3]\n\t"
        "v_max3_i32 %[key], %[key], %[k0], %[k1]\n\t"
        "3:"
        : [v0] "+v"(v0), [v1] "+v"(v1), [v2] "+v"(v2), [v3] "+v"(v3), [f] "+v"(f), [h1] "+v"(h1),
          [key] "+v"(key), [m0] "=&v"(m0), [m1] "=&v"(m1), [m2] "=&v"(m2),
          [m3] "=&v"(m3), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),
          [x0] "=&v"(x0), [x1] "=&v"(x1), [x2] "=&v"(x2), [x3] "=&v"(x3), [ha] "=&v"(ha),
          [hb] "=&v"(hb), [k0] "=&v"(k0), [k1] "=&v"(k1),
          [pw] "=&v"(pw), [d] "=&v"(d), [tp] "=&v"(tp), [inb] "=&s"(inb), [sat] "=&s"(sat), [slt] "=&s"(slt),
          [st] "=&s"(st)
        : [q] "v"(q), [plo] "v"(plo), [phi] "v"(phi), [oe] "s"(oe), [ed] "s"(ed),
          [glo] "s"(glo), [gsp] "s"(gsp), [gfa] "s"(gfa), [gfn] "s"(gfn), [beg] "v"(beg),
          [span] "v"(span), [endv] "v"(beg + span), [gua] "s"(gua), [gun] "s"(gun), [bs] "s"(bs),
          [usp] "s"(usp), [g] "i"(G), [j0] "i"(4 * G), [j1] "i"(4 * G + 1),
          [j2] "i"(4 * G + 2), [j3] "i"(4 * G + 3), [s0] "s"(4 * G), [s1] "s"(4 * G + 1),
          [s2] "s"(4 * G + 2), [s3] "s"(4 * G + 3)
        : "vcc", "scc");
}

template <int G, int QMAX, int SM, bool SYM>
__device__ __forceinline__ void lane_group(uint32_t (&eh)[QMAX + 1], const uint32_t (&q4)[QMAX / 4],
                                           uint2 pr, int beg, int end, int &f, int &h1, int &key,
                                           int &lp1, const LaneRow &r, const LaneCx &c)
{
    constexpr int J0 = 4 * G;
    if constexpr (SM == 1 && SYM && J0 + 3 < QMAX) {
        // skip / fast / masked decided inside the asm on SGPR group bounds
        lane_group_asm<G>(eh[J0], eh[J0 + 1], eh[J0 + 2], eh[J0 + 3], q4[G], pr.x, pr.y, f, h1,
                          key, c.oe_del, c.e_del, r.glo, r.gsp, r.gfa, r.gfn, r.gua, r.gun, r.fast_lo,
                          r.usp, beg, end - beg);
        return;
    }
    if (J0 + 3 < r.ulo || J0 > r.uhi) return;            // uniform skip
    uint32_t pw = 0;
    if constexpr (J0 < QMAX) pw = __builtin_amdgcn_perm(pr.y, pr.x, q4[G]);
    if constexpr (J0 + 3 < QMAX) {
        if (J0 >= r.fast_lo && J0 + 3 < r.fast_hi) {    // uniform: all lanes in band
            lane_cell<J0 + 0, SM, SYM, QMAX + 1>(eh, (int)(int8_t)(pw), f, h1, key, lp1, c);
            lane_cell<J0 + 1, SM, SYM, QMAX + 1>(eh, (int)(int8_t)(pw >> 8), f, h1, key, lp1, c);
            lane_cell<J0 + 2, SM, SYM, QMAX + 1>(eh, (int)(int8_t)(pw >> 16), f, h1, key, lp1, c);
            lane_cell<J0 + 3, SM, SYM, QMAX + 1>(eh, (int)(int8_t)(pw >> 24), f, h1, key, lp1, c);
            return;
        }
    }
    lane_col_masked<J0 + 0, QMAX, SM, SYM>(eh, (int)(int8_t)(pw), beg, end, f, h1, key, lp1, r, c);
    if constexpr (J0 + 1 <= QMAX) lane_col_masked<J0 + 1, QMAX, SM, SYM>(eh, (int)(int8_t)(pw >> 8), beg, end, f, h1, key, lp1, r, c);
    if constexpr (J0 + 2 <= QMAX) lane_col_masked<J0 + 2, QMAX, SM, SYM>(eh, (int)(int8_t)(pw >> 16), beg, end, f, h1, key, lp1, r, c);
    if constexpr (J0 + 3 <= QMAX) lane_col_masked<J0 + 3, QMAX, SM, SYM>(eh, (int)(int8_t)(pw >> 24), beg, end, f, h1, key, lp1, r, c);
}

template <int QMAX, int SM, bool SYM, int... G>
__device__ __forceinline__ void lane_row(std::integer_sequence<int, G...>, uint32_t (&eh)[QMAX + 1],
                                         const uint32_t (&q4)[QMAX / 4], uint2 pr, int beg, int end,
                                         int &f, int &h1, int &key, int &lp1, const LaneRow &r,
                                         const LaneCx &c)
{
    (lane_group<G, QMAX, SM, SYM>(eh, q4, pr, beg, end, f, h1, key, lp1, r, c), ...);
}

// Lazy last-positive column: end_{i+1} = min(lastH + 3, i + w + 2, qlen) needs
// lastH = last j with H(i,j) > 0.  When H(i, end-1) > 0 (the chain value h1 at row end) that is
// end - 1 and nothing is scanned; otherwise the lanes that need it scan the stored row
// eh[j+1].h = H(i,j) right to left from their end - 1 and stop at the first positive cell
// (one exists: m > 0).  Groups above every lane's end and groups after all lanes found one are
// skipped by uniform tests.
template <int QMAX, int GG>
__device__ __forceinline__ bool lastpos_group(const uint32_t (&eh)[QMAX + 1], int end, bool pending,
                                              int &lp1, int gstart)
{
    if (GG > gstart) return pending;                      // uniform
    if (__ballot(pending) == 0) return false;             // uniform
#pragma unroll
    for (int k = 3; k >= 0; --k) {
        const int j = 4 * GG + k;
        if (j < QMAX) {                                   // branch-free selects
            const bool hit = pending & (j < end) & ((eh[j + 1] & 0xffffu) != 0u);
            lp1 = hit ? j + 1 : lp1;
            pending = pending & !hit;
        }
    }
    return pending;
}

template <int QMAX, int... G>
__device__ __forceinline__ void lane_lastpos(std::integer_sequence<int, G...>,
                                             const uint32_t (&eh)[QMAX + 1], int end, bool need,
                                             int &lp1, int gstart)
{
    bool pending = need;
    ((pending = lastpos_group<QMAX, QMAX / 4 - G>(eh, end, pending, lp1, gstart)), ...);
}

constexpr int kTChunkDw = 17;            // dwords per lane per 64-row target chunk

template <int QMAX, int SM, bool SYM>
__global__ __launch_bounds__(64, 2) void lane_kernel(const KParams kp, const int32_t w,
                                                      SeqPair *__restrict__ pairs,
                                                      const int32_t *__restrict__ order,
                                                      const int32_t n,
                                                      const uint8_t *__restrict__ ref,
                                                      const uint8_t *__restrict__ qer,
                                                      int32_t *__restrict__ err)
{
    constexpr int NG = QMAX / 4;        // query words (4 codes each)
    __shared__ uint32_t s_tgt[1][2][kTChunkDw][64];   // 8.7 KB: one wave per workgroup (as pc_kernel)
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = gid < n;
    const int idx = valid ? (order ? order[gid] : gid) : 0;
    SeqPair *sp = pairs + idx;
    int idr = 0, idq = 0, tlen = 0, qlen = 0, h0 = 0;
    if (valid) {
        idr = sp->idr; idq = sp->idq; tlen = sp->len1; qlen = sp->len2; h0 = sp->h0;
        if (qlen > QMAX || qlen < 0 || tlen < 0 || h0 < 0 ||
            (int64_t)h0 + (int64_t)kp.maxsc * min(qlen, tlen) >= 32768) {   // int16 cells
            atomicOr(err, 1);
            valid = false;
        }
    }
    // query codes -> perm selectors (4 per VGPR).  Aligned dword loads (a dword holding at
    // least one byte of the query never leaves that byte's page), all issued before use;
    // bytes are realigned with v_alignbyte.  Codes must be 0..4 (upstream contract).
    uint32_t q4[NG];
    {
        uint32_t wv[NG + 1];
        const uintptr_t qa = (uintptr_t)(qer + idq);
        const uint32_t *wp = (const uint32_t *)(qa & ~(uintptr_t)3);
        const int sh = (int)(qa & 3);
        const int nw = (valid && qlen > 0) ? (sh + qlen + 3) >> 2 : 0;
        if (nw > 0) {
#pragma unroll
            for (int g = 0; g <= NG; ++g) wv[g] = wp[min(g, nw - 1)];
        } else {
#pragma unroll
            for (int g = 0; g <= NG; ++g) wv[g] = 0;
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) q4[g] = __builtin_amdgcn_alignbyte(wv[g + 1], wv[g], sh);
    }
    // A.1 first row: eh[j].h = max(h0 - oe_ins - (j-1) e_ins, 0), 1 <= j <= qlen
    uint32_t eh[QMAX + 1];
    const int oe_ins = kp.o_ins + kp.e_ins;
    eh[0] = (uint32_t)h0;
#pragma unroll
    for (int j = 1; j <= QMAX; ++j) eh[j] = (j <= qlen) ? (uint32_t)max(h0 - oe_ins - (j - 1) * kp.e_ins, 0) : 0u;
    // A.2 per-lane band cap, integer form of (int)((double)N / e + 1.)
    int wl = w;
    {
        const int ni = qlen * kp.maxsc + kp.end_bonus - kp.o_ins;
        const int nd = qlen * kp.maxsc + kp.end_bonus - kp.o_del;
        wl = min(wl, max((ni + kp.e_ins) / kp.e_ins, 1));
        wl = min(wl, max((nd + kp.e_del) / kp.e_del, 1));
    }
    // A.3 state
    int best = h0, best_i = -1, best_j = -1, max_ie = -1, gsc = -1, moff = 0, endc = qlen;
    bool alive = valid && tlen > 0;
    // Target bases stream HBM -> LDS by LDS-DMA (global_load_lds_dword), no VGPRs involved:
    // per wave two chunk buffers of 64 rows (17 aligned dwords per lane, layout [dword][lane]
    // so each DMA instruction writes 256 contiguous bytes).  Chunk c covers rows
    // [64c, 64c + 64) = dwords [16c, 16c + 17) of the lane's aligned window; it is issued one
    // chunk ahead and waited for once (vmcnt) at its first row.  A dword holding >= 1 byte of
    // the window never leaves that byte's page, so clamped aligned loads are always safe.
    const uint8_t *tp = ref + idr;
    const int tsh = (int)((uintptr_t)tp & 3);
    const uint32_t *twp = (const uint32_t *)(tp - tsh);
    const int tlast = max((tsh + tlen - 1) >> 2, 0);      // last dword holding a valid byte
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    auto issue_chunk = [&](int ch) {
        uint32_t *dst = &s_tgt[wv][ch & 1][0][0];
#pragma unroll
        for (int k = 0; k < kTChunkDw; ++k)
            __builtin_amdgcn_global_load_lds((gptr_t)(twp + min(16 * ch + k, tlast)),
                                             (lptr_t)(dst + 64 * k), 4, 0, 0);
    };
    if (alive) { issue_chunk(0); issue_chunk(1); }
    uint32_t tcur = 0;
    const int wl_max = wave_max(alive ? wl : -1);
    const int wl_min = wave_min(alive ? wl : INT_MAX);
    const LaneCx cx{kp.e_del, kp.o_del + kp.e_del, kp.e_ins, kp.o_ins + kp.e_ins, kp.maxsc};

    for (int i = 0;; ++i) {
        const bool act = alive && i < tlen;
        alive = act;
        if (__ballot(act) == 0) break;
        const int beg = max(0, i - wl);
        const int end = min(min(endc, i + wl + 1), qlen);
        endc = end;
        // uniform pass bounds: fast = [beg_u, min end) when every live lane shares beg,
        // edge = [fast_hi, max end] (or the whole [min beg, max end] otherwise)
        const int emax = wave_max(act ? end : -1);
        const int emin = wave_min(act ? end : INT_MAX);
        LaneRow r;
        r.ulo = __builtin_amdgcn_readfirstlane(max(0, i - wl_max));      // min beg (live lanes)
        r.uhi = __builtin_amdgcn_readfirstlane(emax);                    // max end
        r.fast_lo = __builtin_amdgcn_readfirstlane(max(0, i - wl_min));  // max beg
        r.fast_hi = __builtin_amdgcn_readfirstlane(emin);                // min end
        r.glo = r.ulo >> 2;
        r.gsp = max((r.uhi >> 2) - r.glo, -1);      // -1 (as unsigned: huge) never happens: uhi >= ulo
        r.gfa = (r.fast_lo + 3) >> 2;
        r.gfn = max((r.fast_hi >> 2) - r.gfa, 0);
        {   // U groups: left edge uniform (every lane's beg == fast_lo) or no cell left of it,
            // and right edge uniform or every cell < fast_hi
            const int gl = (r.ulo == r.fast_lo) ? 0 : r.gfa;
            const int gr = (r.uhi == r.fast_hi) ? 64 : (r.fast_hi >> 2);
            r.gua = gl;
            r.gun = max(gr - gl, 0);
            r.usp = r.fast_hi - r.fast_lo;
        }
        if (act) {
            if ((i & 3) == 0) {            // new 4-row block: 4 target bases from LDS
                if ((i & 63) == 0) {          // chunk boundary: its DMA was issued 64 rows ago
                    __builtin_amdgcn_s_waitcnt(0x0F70);      // vmcnt(0)
                    __builtin_amdgcn_sched_barrier(0);
                }
                const int k = (i >> 2) & 15;
                const uint32_t *src = &s_tgt[wv][(i >> 6) & 1][k][ln];
                tcur = __builtin_amdgcn_alignbyte(src[64], src[0], tsh);
                if ((i & 63) == 0) {
                    __builtin_amdgcn_sched_barrier(0);
                    if (i > 0) issue_chunk((i >> 6) + 1);   // refill the buffer just drained
                }
            }
            // per-row score profile of target base t (8 bytes: mat[t][q], q = 0..7)
            const uint32_t t = (tcur >> (8 * (i & 3))) & 0xffu;
            uint2 pr = make_uint2(kp.prof[4][0], kp.prof[4][1]);
            pr = (t == 3) ? make_uint2(kp.prof[3][0], kp.prof[3][1]) : pr;
            pr = (t == 2) ? make_uint2(kp.prof[2][0], kp.prof[2][1]) : pr;
            pr = (t == 1) ? make_uint2(kp.prof[1][0], kp.prof[1][1]) : pr;
            pr = (t == 0) ? make_uint2(kp.prof[0][0], kp.prof[0][1]) : pr;
            int h1 = (beg == 0) ? max(h0 - (kp.o_del + kp.e_del * (i + 1)), 0) : 0;
            int f = 0, key = -1, lp1 = 0;
            // wave priority as in pc_kernel: the row's serial scalar chain at 2,
            // the group sequence at 0
            __builtin_amdgcn_s_setprio(0);
            lane_row<QMAX, SM, SYM>(std::make_integer_sequence<int, QMAX / 4 + 1>{}, eh, q4, pr,
                                    beg, end, f, h1, key, lp1, r, cx);
            __builtin_amdgcn_s_setprio(2);
            const int m = key >> 16, mj = key & 0xffff;
            if (end == qlen) {                    // A.4: j == qlen (beg <= end always)
                if (!(gsc > h1)) max_ie = i;
                gsc = max(gsc, h1);
            }
            if (m <= 0) {
                alive = false;
            } else if (m > best) {
                best = m; best_i = i; best_j = mj;
                moff = max(moff, abs(mj - i));
            } else if (kp.zdrop > 0) {
                const int di = i - best_i, dj = mj - best_j;
                const int dz = (di > dj) ? best - m - (di - dj) * kp.e_del
                                         : best - m - (dj - di) * kp.e_ins;
                if (dz > kp.zdrop) alive = false;
            }
            if (alive) {                           // end_{i+1} = min(lastH + 3, ...), DESIGN.md §3
                if constexpr (SM == 1 && SYM) {    // asm groups: lastH recovered lazily
                    const bool need = h1 == 0;     // H(i, end-1) == 0 -> lastH < end - 1
                    if (__ballot(need)) {
                        lp1 = 0;
                        lane_lastpos<QMAX>(std::make_integer_sequence<int, QMAX / 4 + 1>{}, eh, end, need,
                                           lp1, (emax - 1) >> 2);
                    }
                    endc = min((need ? lp1 : end) + 2, qlen);
                } else {
                    endc = min(lp1 + 2, qlen);     // C++ cells track lp1 = 1 + lastH
                }
            }
        }
    }
    if (valid) {
        sp->score = best;
        sp->tle = best_i + 1;
        sp->gtle = max_ie + 1;
        sp->qle = best_j + 1;
        sp->gscore = gsc;
        sp->max_off = moff;
    }
}

// ------------------------------------------------------------------ wide kernel
// Literal A.4 per lane (int32 cells, narrowing loops as written), eh in HBM scratch at
// scratch[j * stride + slot] so that lanes of a wave touching the same column coalesce.
__global__ __launch_bounds__(256) void wide_kernel(const KParams kp, const int32_t w,
                                                   SeqPair *__restrict__ pairs,
                                                   const int32_t *__restrict__ order,
                                                   const int32_t n,
                                                   const uint8_t *__restrict__ ref,
                                                   const uint8_t *__restrict__ qer,
                                                   int2 *__restrict__ scratch,
                                                   const int32_t stride)
{
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= n) return;
    const int idx = order ? order[gid] : gid;
    SeqPair *sp = pairs + idx;
    const int tlen = sp->len1, qlen = sp->len2, h0 = sp->h0;
    const uint8_t *query = qer + sp->idq, *target = ref + sp->idr;
    int2 *eh = scratch + gid;
#define EH(j) eh[(int64_t)(j) * stride]
    const int oe_del = kp.o_del + kp.e_del, oe_ins = kp.o_ins + kp.e_ins;
    for (int j = 0; j <= qlen + 1; ++j) EH(j) = make_int2(0, 0);
    EH(0).x = h0;
    EH(1).x = h0 > oe_ins ? h0 - oe_ins : 0;
    for (int j = 2; j <= qlen && EH(j - 1).x > kp.e_ins; ++j) EH(j).x = EH(j - 1).x - kp.e_ins;
    int wl = w;
    {
        const int ni = qlen * kp.maxsc + kp.end_bonus - kp.o_ins;
        const int nd = qlen * kp.maxsc + kp.end_bonus - kp.o_del;
        wl = min(wl, max((ni + kp.e_ins) / kp.e_ins, 1));
        wl = min(wl, max((nd + kp.e_del) / kp.e_del, 1));
    }
    int best = h0, best_i = -1, best_j = -1, max_ie = -1, gsc = -1, moff = 0;
    int beg = 0, end = qlen;
    for (int i = 0; i < tlen; ++i) {
        int f = 0, h1, m = 0, mj = -1, j;
        const int8_t *row = kp.mat + 5 * min((int)target[i], 4);
        if (beg < i - wl) beg = i - wl;
        if (end > i + wl + 1) end = i + wl + 1;
        if (end > qlen) end = qlen;
        h1 = (beg == 0) ? max(h0 - (kp.o_del + kp.e_del * (i + 1)), 0) : 0;
        for (j = beg; j < end; ++j) {
            int2 p = EH(j);
            int M = p.x, e = p.y, h;
            p.x = h1;
            M = M ? M + row[min((int)query[j], 4)] : 0;
            h = max3i(M, e, f);
            h1 = h;
            mj = m > h ? mj : j;
            m = m > h ? m : h;
            e = max(e - kp.e_del, max(M - oe_del, 0));
            p.y = e;
            EH(j) = p;
            f = max(f - kp.e_ins, max(M - oe_ins, 0));
        }
        EH(end) = make_int2(h1, 0);
        if (j == qlen) {
            max_ie = gsc > h1 ? max_ie : i;
            gsc = gsc > h1 ? gsc : h1;
        }
        if (m == 0) break;
        if (m > best) {
            best = m; best_i = i; best_j = mj;
            moff = max(moff, abs(mj - i));
        } else if (kp.zdrop > 0) {
            const int di = i - best_i, dj = mj - best_j;
            const int dz = (di > dj) ? best - m - (di - dj) * kp.e_del : best - m - (dj - di) * kp.e_ins;
            if (dz > kp.zdrop) break;
        }
        for (j = beg; j < end; ++j) { const int2 p = EH(j); if (p.x || p.y) break; }
        beg = j;
        for (j = end; j >= beg; --j) { const int2 p = EH(j); if (p.x || p.y) break; }
        end = min(j + 2, qlen);
    }
#undef EH
    sp->score = best;
    sp->tle = best_i + 1;
    sp->gtle = max_ie + 1;
    sp->qle = best_j + 1;
    sp->gscore = gsc;
    sp->max_off = moff;
}

// ------------------------------------------------------------------ launchers
template <int QMAX>
static hipError_t launch_lane_q(const KParams &kp, int32_t w, SeqPair *pairs, const int32_t *order,
                                int32_t n, const uint8_t *ref, const uint8_t *qer, int32_t *err,
                                hipStream_t s)
{
    const dim3 block(64), grid((unsigned)((n + 63) / 64));
    const bool sym = kp.o_del == kp.o_ins && kp.e_del == kp.e_ins;
    if (kp.maxsc == 1 && sym)
        hipLaunchKernelGGL((lane_kernel<QMAX, 1, true>), grid, block, 0, s, kp, w, pairs, order, n, ref, qer, err);
    else
        hipLaunchKernelGGL((lane_kernel<QMAX, 2, false>), grid, block, 0, s, kp, w, pairs, order, n, ref, qer, err);
    return hipGetLastError();
}

hipError_t launch_lane_kernel(int qmax, const KParams &kp, int32_t w, SeqPair *pairs,
                              const int32_t *order, int32_t n, const uint8_t *ref,
                              const uint8_t *qer, int32_t *err, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    switch (qmax) {
#ifndef BSW_ONLY_Q160
    case 32: return launch_lane_q<32>(kp, w, pairs, order, n, ref, qer, err, s);
    case 64: return launch_lane_q<64>(kp, w, pairs, order, n, ref, qer, err, s);
    case 96: return launch_lane_q<96>(kp, w, pairs, order, n, ref, qer, err, s);
    case 128: return launch_lane_q<128>(kp, w, pairs, order, n, ref, qer, err, s);
#endif
    case 160: return launch_lane_q<160>(kp, w, pairs, order, n, ref, qer, err, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_wide_kernel(const KParams &kp, int32_t w, SeqPair *pairs, const int32_t *order,
                              int32_t n, const uint8_t *ref, const uint8_t *qer, int2 *scratch,
                              int32_t scratch_stride, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(wide_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, kp, w,
                       pairs, order, n, ref, qer, scratch, scratch_stride);
    return hipGetLastError();
}

}  // namespace bsw
