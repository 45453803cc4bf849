// bsw_pc.hip -- the packed-COLUMN lane kernel for gfx950: one SeqPair per
// lane as in the lane kernel (bsw_kernels.hip), but the pair's DP row is split into an H plane
// and an E plane, each packed TWO COLUMNS per VGPR, so that every column-independent step of
// the ksw_extend2 recurrence is one v_pk_* instruction for two cells.
//
//   HH[k] = {H(i-1, 2k-1), H(i-1, 2k)}   -- "slot" s holds eh[s].h = H(i-1, s-1), the hold of column s
//   EE[k] = {E(i, 2k),     E(i, 2k+1)}   -- eh[s].e
//   Q[g]  = query codes of columns 4g..4g+3 in byte order {c0, c2, c1, c3}
//
// Per 4-column group (two HH and two EE registers), default scoring (match 1, one mismatch
// value, N -1, symmetric gaps; the host's pk_ok contract):
//   scores   : Y = v_perm(profile[t], Q[g]) -> {S0, S2, S1, S3} bytes; {S0, S1} and {S2, S3}
//              sign-extended by packed 16-bit shifts                         (4 instructions)
//   phase 1  : M = hold + min(S, hold) (the A.5 gate), T~ = M - oe, ME = max(M, E),
//              E' = max(E - e, T~) -- 6 packed instructions per 2 columns     (12)
//   F chain  : h = max(F, ME_j), F = max(sat(F - e), T~_j) per column, 32-bit ops with SDWA
//              word selects                                                   (12)
//   pack/key : HH <- {h_{j-1}, h_j} (v_lshl_or), key = max(HH << 8 | j) by v_pk_max_u16 (6)
// = 34 VALU per 4 cells, against 47 for the lane kernel's fast group.  ~200 VGPRs at
// QMAX = 160: two waves per SIMD (the occupancy the packed two-pairs-per-lane kernel lacks).
//
// Eligibility (planner, bsw_host.cpp): pk_ok scoring, h0 + min(qlen, tlen) <= 255 (H <= 255:
// the 8-bit key H << 8 | j and the 16-bit lanes), qlen < QMAX (slot qlen inside a group).
//
// Band edges (per lane [beg, end)): a group is FAST when every live lane has all
// four columns in band and 4G > beg (so the entering F / H chain is valid); otherwise it is
// MASKED: the same arithmetic, then per-lane packed masks write slots <= end only (slots
// beyond end keep their stale values, A.7: a later row whose end grows by 2 reads them), put
// E = 0 at slot end, drop slots > end (and < beg) from the key, and pass H(i, end-1) along the
// chain (h1 at row end = H(i, end-1), for gscore and the lazy last-positive scan).  Groups that
// contain some lane's beg also reset F and H to 0 entering column beg.  Slots left of beg may
// take garbage: they are never read again (beg never decreases).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <limits.h>
#include <utility>
#include "bsw_kernels.h"
#include "bsw_wave.h"

namespace bsw {

constexpr int kPcChunkDw = 17;           // dwords per lane per 64-row target chunk (as lane kernel)
#ifndef BSW_PC_EXP_HALFHEAD
#define BSW_PC_EXP_HALFHEAD 0
#endif
#ifdef BSW_PC_STATS
__device__ unsigned long long g_pc_stats[8];
// per-wave schedule record (tools/pc_times.py): start / end (s_memrealtime, 100 MHz), XCC id and
// HW_ID (CU / SIMD / SE), rows run -- the launch's occupancy over time, ramp-up and tail
constexpr int kPcTimesMax = 1 << 16;
__device__ unsigned long long g_pc_times[kPcTimesMax][4];
#endif

struct PcRow {                           // per-row uniform (SGPR) group sets, bit G = group G
    uint64_t enter;                      // groups touching slots [min beg, max end]
    uint64_t fast;                       // FAST groups
    uint64_t left;                       // groups containing some lane's beg (masked-L)
};

// groups lo .. lo + n - 1 as a bit set (uniform; only bits < QMAX / 4 <= 40 are read).  Callers
// pass n >= 0 and lo < 40 whenever n > 0 (lo: a live lane's group; the FAST set's lo may pass 63
// only with n == 0), so a width clamped to 63 and one s_bfm_b64 give every bit that is read --
// no branches in the row's scalar chain
__device__ __forceinline__ uint64_t gbits(int lo, int n)
{
    uint64_t m;
    asm("s_bfm_b64 %0, %1, %2" : "=s"(m)
        : "s"(__builtin_amdgcn_readfirstlane(min(n, 63))), "s"(__builtin_amdgcn_readfirstlane(lo)));
    return m;
}

// {v, v} as two int16 halves
__device__ __forceinline__ uint32_t pack2(int v) { return ((uint32_t)v & 0xffffu) * 0x10001u; }

#define PC_SDWA(op, d, a, b, sel) \
    op "_sdwa " d ", " a ", " b " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" sel "\n\t"

// phase 1 of one packed register X (columns 2k, 2k+1): S in %[sX] -> M -> ME; T~ in %[tX];
// E~' into EOUT (in place for FAST, %[xX] for MASKED).
//
// T and E are kept UNCLAMPED (T~ = M - oe, E~' = max(E~ - e, T~)): only their positive parts
// matter.  Invariant max(E~, 0) = E: E' = max(E - e, T) = max(max(E~, 0) - e, T~, 0) =
// max(E~ - e, T~, 0) (as -e < 0).  The F chain clamps instead (f - e saturates at 0, so
// F >= 0 always) and H = max(ME, F) = max(M, E~, F) equals max(M, E, F) because F >= 0.
// Bounds: M >= -127, oe < 4096 (pk_ok), so T~, E~ stay far inside int16.
#define PC_PH1_(X, EOUT, ESUB)                                                          \
    "v_pk_min_i16 %[s" X "], %[s" X "], %[h" X "]\n\t"                                      \
    "v_pk_add_u16 %[s" X "], %[s" X "], %[h" X "]\n\t"                                      \
    "v_pk_sub_i16 %[t" X "], %[s" X "], %[oe2]\n\t"                                         \
    "v_pk_max_i16 %[s" X "], %[s" X "], %[e" X "]\n\t"                                      \
    ESUB                                                                                     \
    "v_pk_max_i16 " EOUT ", " EOUT ", %[t" X "]\n\t"
#define PC_PH1(X, EOUT) PC_PH1_(X, EOUT, "v_pk_sub_i16 " EOUT ", %[e" X "], %[ed2]\n\t")
// byte planes (BY kernels): E enters >= 0 (a stored byte), so E - e saturating at 0 makes E'
// = max(sat(E - e), T~) = max(E - e, T, 0) clamped for free -- a byte again
#define PC_PH1B(X, EOUT) PC_PH1_(X, EOUT, "v_pk_sub_u16 " EOUT ", %[e" X "], %[ed2] clamp\n\t")

#define PC_SCORES                                                                        \
    "v_perm_b32 %[y], %[phi], %[plo], %[q]\n\t"                                              \
    "v_pk_lshlrev_b16 %[sa], 8, %[y] op_sel_hi:[0,1]\n\t"                                    \
    "v_pk_ashrrev_i16 %[sa], 8, %[sa] op_sel_hi:[0,1]\n\t"                                   \
    "v_pk_ashrrev_i16 %[sb], 8, %[y] op_sel_hi:[0,1]\n\t"

// one F-chain cell: H -> C, F updated.  X = a|b register, W = WORD_0|WORD_1 half
// ME and T~ may be negative now: their word selects must sign-extend (sext)
#define PC_CELL(C, X, W)                                                                 \
    PC_SDWA("v_max_i32", C, "%[f]", "sext(%[s" X "])", W)                                    \
    "v_subrev_u32_e64 %[f], %[ed], %[f] clamp\n\t"                                           \
    PC_SDWA("v_max_i32", "%[f]", "%[f]", "sext(%[t" X "])", W)

// masked cell: optional reset entering column J (J == beg: F = 0, H(i, J-1) = 0), then the
// cell, then C = (J < end) ? H : HP (H(i, end-1) travels on past end)
#define PC_RESET(HP, RJ)                                                                 \
    "v_cmp_ne_u32_e32 vcc, " RJ ", %[begv]\n\t"                                              \
    "v_cndmask_b32_e32 " HP ", 0, " HP ", vcc\n\t"                                           \
    "v_cndmask_b32_e32 %[f], 0, %[f], vcc\n\t"
#define PC_MCELL(C, HP, X, W, J)                                                         \
    PC_CELL(C, X, W)                                                                         \
    "v_cmp_lt_i32_e32 vcc, " J ", %[endv]\n\t"                                               \
    "v_cndmask_b32_e32 " C ", " HP ", " C ", vcc\n\t"

// masked write-back of register X from packed new values in %[pX]:
//   slot <= end : HH <- new (else stale kept);  slot < end : EE <- E';  slot == end : EE <- 0
//   key over slots in [beg, end] (LEFT adds the slot >= beg mask)
#define PC_MWRITE(X, KEYSRC, LEFT)                                                       \
    "v_pk_sub_i16 %[y], %[jj" X "], %[endw]\n\t"                                             \
    "v_pk_ashrrev_i16 %[y], 15, %[y] op_sel_hi:[0,1]\n\t"                                    \
    "v_bfi_b32 %[h" X "], %[y], %[p" X "], %[h" X "]\n\t"                                    \
    "v_bfi_b32 %[e" X "], %[y], 0, %[e" X "]\n\t"                                            \
    KEYSRC                                                                                   \
    "v_and_b32_e32 %[p" X "], %[p" X "], %[y]\n\t"                                           \
    "v_pk_sub_i16 %[y], %[jj" X "], %[endm1w]\n\t"                                           \
    "v_pk_ashrrev_i16 %[y], 15, %[y] op_sel_hi:[0,1]\n\t"                                    \
    "v_bfi_b32 %[e" X "], %[y], %[x" X "], %[e" X "]\n\t"                                    \
    LEFT                                                                                     \
    "v_pk_max_u16 %[key], %[key], %[p" X "]\n\t"
#define PC_LEFTMASK(X)                                                                   \
    "v_pk_sub_i16 %[y], %[begm2w], %[jj" X "]\n\t"                                           \
    "v_pk_ashrrev_i16 %[y], 15, %[y] op_sel_hi:[0,1]\n\t"                                    \
    "v_and_b32_e32 %[p" X "], %[p" X "], %[y]\n\t"

// masked body (chain variant CH), shared by the L (left-reset) and R forms
#define PC_MASKED(CH0, CH1, CH2, CH3, KA, KB, LA, LB) PC_MASKED_(PC_PH1, CH0, CH1, CH2, CH3, KA, KB, LA, LB)
#define PC_MASKED_(PH, CH0, CH1, CH2, CH3, KA, KB, LA, LB)                               \
    PH("a", "%[xa]") PH("b", "%[xb]")                                                        \
    CH0 CH1                                                                                  \
    "v_lshl_or_b32 %[pa], %[c0], 16, %[h1]\n\t"                                              \
    CH2 CH3                                                                                  \
    "v_lshl_or_b32 %[pb], %[c2], 16, %[c1]\n\t"                                              \
    PC_MWRITE("a", KA, LA) PC_MWRITE("b", KB, LB)

#ifdef BSW_PC_STATS          // group-path counters (tools/pc_stats.py; never in the product build)
#define PC_CNT(k) "v_add_u32_e32 %[ct" #k "], 1, %[ct" #k "]\n\t"
#define PC_CNT_OPS , [ct0] "+v"(ctr[0]), [ct1] "+v"(ctr[1]), [ct2] "+v"(ctr[2]), [ct3] "+v"(ctr[3])
#else
#define PC_CNT(k)
#define PC_CNT_OPS
#endif

// FAST F chain, packed (two columns per instruction where the recurrence allows it).
// F(j+1) = max(sat(F(j) - e), T~(j)); H(j) = max(ME(j), F(j)).  Per register X (columns 2k, 2k+1)
// with Fp = {F(2k), sat(F(2k) - e)} entering:
//   Fp <- max(Fp, {T~(2k), T~(2k)})          = {max(F(2k), T~(2k)), F(2k+1)}  (the low half may
//                                              absorb T~(2k): ME >= M > T~, so H(2k) is unchanged)
//   Hp  = max(Fp, ME)                        = {H(2k), H(2k+1)}
//   Fp <- max(sat({F(2k+1) - e, F(2k+1) - 2e}), {T~(2k+1), T~(2k+1) - e})
//                                            = {F(2k+2), sat(F(2k+2) - e)}
// (sat(max(a, b) - e) = max(sat(a - e), sat(b - e)); the second half is >= 0 through its first
// operand, so T~ needs no clamp).  The group enters with a clean f = F(4G) and leaves with a clean
// f = F(4G+4) (32-bit ops for the last step, so masked bodies read it unchanged), and leaves
// h1 = {H(4G+2), H(4G+3)}: h1 travels in its HIGH half between groups, so the new row
// registers are two byte-aligns, HH[2G] = {H(4G-1), H(4G)}, HH[2G+1] = {H(4G+1), H(4G+2)}.
// 10 VALU per 4 cells for the chain (12 before) and 2 for the packing.
#define PC_FAST_CHAIN                                                                    \
    PC_FAST_CHAIN_("v_alignbyte_b32 %[ha], %[pa], %[h1], 2\n\t", "v_alignbyte_b32 %[hb], %[h1], %[pa], 2\n\t")
// A1 reads the entering h1 (H(4G-1) in its high half) and pa = {H(4G), H(4G+1)}; A2 the leaving
// h1 = {H(4G+2), H(4G+3)}: the int16 form builds HH[2G], HH[2G+1]; the byte form (BY) builds
// HB[G] = bytes {H(4G-1), H(4G), H(4G+1), H(4G+2)} by two v_perm (the same instruction count)
#define PC_FAST_CHAIN_(A1, A2)                                                           \
    "v_pk_sub_u16 %[fp], %[f], %[e0e] op_sel_hi:[0,1] clamp\n\t"                            \
    "v_pk_max_i16 %[fp], %[fp], %[ta] op_sel_hi:[1,0]\n\t"                                  \
    "v_pk_max_i16 %[pa], %[fp], %[sa]\n\t"                                                  \
    "v_pk_sub_u16 %[fp], %[fp], %[ee2] op_sel:[1,0] clamp\n\t"                              \
    "v_pk_sub_i16 %[y], %[ta], %[e0e] op_sel:[1,0]\n\t"                                     \
    "v_pk_max_i16 %[fp], %[fp], %[y]\n\t"                                                   \
    A1                                                                                       \
    "v_pk_max_i16 %[fp], %[fp], %[tb] op_sel_hi:[1,0]\n\t"                                  \
    "v_pk_max_i16 %[h1], %[fp], %[sb]\n\t"                                                  \
    "v_sub_u32_sdwa %[f], %[fp], %[ed] clamp dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t" \
    A2                                                                                       \
    PC_SDWA("v_max_i32", "%[f]", "%[f]", "sext(%[tb])", "WORD_1")

// Layout: the FAST body is the fall-through path (one bit test, a not-taken branch, no taken
// branch); skipped and masked groups branch to code in subsection 1 of the kernel's section
// (out of line, after the kernel's main body) and back.  Branch targets stay inside the
// kernel's own section (built with -ffunction-sections), well within s_cbranch's +-128 KB.
#define PC_GROUP_ASM(KEYA_FAST, KEYA_MASK)                                                \
    asm volatile(                                                                            \
        "s_bitcmp1_b64 %[mfa], %[g]\n\t"             /* every live lane in band: FAST */    \
        "s_cbranch_scc0 5f\n\t"                                                              \
        PC_CNT(0) PC_CNT(1)                                                                  \
        PC_SCORES                                                                            \
        PC_PH1("a", "%[ea]") PC_PH1("b", "%[eb]")                                            \
        PC_FAST_CHAIN                                                                        \
        KEYA_FAST                                                                            \
        "v_pk_max_u16 %[key], %[key], %[pa]\n\t"                                             \
        "v_lshl_or_b32 %[pb], %[hb], 8, %[jjb]\n\t"                                          \
        "v_pk_max_u16 %[key], %[key], %[pb]\n"                                               \
        "3:\n"                                                                               \
        ".subsection 1\n"                                                                    \
        "5:\n\t"                                                                             \
        "s_bitcmp1_b64 %[men], %[g]\n\t"             /* outside [min beg, max end]: skip */ \
        "s_cbranch_scc0 3b\n\t"                                                              \
        "s_setprio 2\n\t"                            /* masked bodies: short per-cell chains */\
        PC_CNT(0)                                                                            \
        "v_lshrrev_b32_e32 %[h1], 16, %[h1]\n\t"     /* masked bodies: h1 as a clean int */ \
        PC_SCORES                                                                            \
        "s_bitcmp1_b64 %[mle], %[g]\n\t"             /* some lane's beg in this group: L */ \
        "s_cbranch_scc1 4f\n\t"                                                              \
        PC_CNT(2)                                                                            \
        PC_MASKED(PC_MCELL("%[c0]", "%[h1]", "a", "WORD_0", "%[j0]"),                        \
                  PC_MCELL("%[c1]", "%[c0]", "a", "WORD_1", "%[j1]"),                        \
                  PC_MCELL("%[c2]", "%[c1]", "b", "WORD_0", "%[j2]"),                        \
                  PC_MCELL("%[h1]", "%[c2]", "b", "WORD_1", "%[j3]"),                        \
                  KEYA_MASK, "v_lshl_or_b32 %[pb], %[pb], 8, %[jjb]\n\t", "", "")           \
        "v_lshlrev_b32_e32 %[h1], 16, %[h1]\n\t"                                              \
        "s_setprio 0\n\t"                                                                    \
        "s_branch 3b\n"                                                                      \
        "4:\n\t"                                                                             \
        PC_CNT(3)                                                                            \
        PC_MASKED(PC_RESET("%[h1]", "%[r0]") PC_MCELL("%[c0]", "%[h1]", "a", "WORD_0", "%[j0]"), \
                  PC_RESET("%[c0]", "%[j1]") PC_MCELL("%[c1]", "%[c0]", "a", "WORD_1", "%[j1]"), \
                  PC_RESET("%[c1]", "%[j2]") PC_MCELL("%[c2]", "%[c1]", "b", "WORD_0", "%[j2]"), \
                  PC_RESET("%[c2]", "%[j3]") PC_MCELL("%[h1]", "%[c2]", "b", "WORD_1", "%[j3]"), \
                  KEYA_MASK, "v_lshl_or_b32 %[pb], %[pb], 8, %[jjb]\n\t",                    \
                  PC_LEFTMASK("a"), PC_LEFTMASK("b"))                                        \
        "v_lshlrev_b32_e32 %[h1], 16, %[h1]\n\t"                                              \
        "s_setprio 0\n\t"                                                                    \
        "s_branch 3b\n"                                                                      \
        ".subsection 0\n"                                                                    \
        : [ha] "+v"(ha), [hb] "+v"(hb), [ea] "+v"(ea), [eb] "+v"(eb), [f] "+v"(f),           \
          [h1] "+v"(h1), [key] "+v"(key), [y] "=&v"(y), [sa] "=&v"(sa), [sb] "=&v"(sb),     \
          [ta] "=&v"(ta), [tb] "=&v"(tb), [xa] "=&v"(xa), [xb] "=&v"(xb), [c0] "=&v"(c0),    \
          [c1] "=&v"(c1), [c2] "=&v"(c2), [pa] "=&v"(pa), [pb] "=&v"(pb), [fp] "=&v"(fp)    \
          PC_CNT_OPS                                                                         \
        : [q] "v"(q), [plo] "v"(plo), [phi] "v"(phi), [oe2] "s"(oe2), [ed2] "s"(ed2),        \
          [ed] "s"(ed), [e0e] "s"(e0e), [ee2] "s"(ee2), [men] "s"(r.enter), [mfa] "s"(r.fast), [mle] "s"(r.left),           \
          [endw] "v"(endw), [endm1w] "v"(endm1w),                                            \
          [begm2w] "v"(begm2w), [endv] "v"(endv), [begv] "v"(begv), [g] "i"(G),             \
          [jja] "s"(JJA), [jjb] "s"(JJB), [j0] "i"(4 * G), [j1] "i"(4 * G + 1),              \
          [j2] "i"(4 * G + 2), [j3] "i"(4 * G + 3), [r0] "i"(R0)                             \
        : "vcc", "scc")

// BSW_PC_JKEY (default 1): the FAST key from ONE scalar constant per group instead of two.  The
// key halves H << 8 | j (H <= 255 in this kernel's regime) are built by v_perm from the group's
// four column numbers as BYTES of one SGPR, J4 = {4G-1, 4G, 4G+1, 4G+2}, with two loop-invariant
// VGPR selectors (gfx9 VOP3 reads one SGPR): one s_mov per group instead of two for the packed
// {4G-1, 4G} / {4G+1, 4G+2} constants of v_lshl_or -- 24 fewer SALU on a C2 row.  The masked
// bodies (out of line, ~9% of groups) load those packed constants themselves (two s_mov there).
#ifndef BSW_PC_JKEY
#define BSW_PC_JKEY 1
#endif
#define PC_GROUP_ASM_J                                                                   \
    asm volatile(                                                                            \
        "s_bitcmp1_b64 %[mfa], %[g]\n\t"                                                     \
        "s_cbranch_scc0 5f\n\t"                                                              \
        PC_CNT(0) PC_CNT(1)                                                                  \
        PC_SCORES                                                                            \
        PC_PH1("a", "%[ea]") PC_PH1("b", "%[eb]")                                            \
        PC_FAST_CHAIN                                                                        \
        "v_perm_b32 %[pa], %[ha], %[j4], %[ska]\n\t"                                         \
        "v_pk_max_u16 %[key], %[key], %[pa]\n\t"                                             \
        "v_perm_b32 %[pb], %[hb], %[j4], %[skb]\n\t"                                         \
        "v_pk_max_u16 %[key], %[key], %[pb]\n"                                               \
        "3:\n"                                                                               \
        ".subsection 1\n"                                                                    \
        "5:\n\t"                                                                             \
        "s_bitcmp1_b64 %[men], %[g]\n\t"                                                     \
        "s_cbranch_scc0 3b\n\t"                                                              \
        "s_setprio 2\n\t"                                                                    \
        PC_CNT(0)                                                                            \
        "s_mov_b32 %[jja], %[ija]\n\t"               /* packed {4G-1, 4G}, {4G+1, 4G+2} */ \
        "s_mov_b32 %[jjb], %[ijb]\n\t"                                                       \
        "v_lshrrev_b32_e32 %[h1], 16, %[h1]\n\t"                                             \
        PC_SCORES                                                                            \
        "s_bitcmp1_b64 %[mle], %[g]\n\t"                                                     \
        "s_cbranch_scc1 4f\n\t"                                                              \
        PC_CNT(2)                                                                            \
        PC_MASKED(PC_MCELL("%[c0]", "%[h1]", "a", "WORD_0", "%[j0]"),                        \
                  PC_MCELL("%[c1]", "%[c0]", "a", "WORD_1", "%[j1]"),                        \
                  PC_MCELL("%[c2]", "%[c1]", "b", "WORD_0", "%[j2]"),                        \
                  PC_MCELL("%[h1]", "%[c2]", "b", "WORD_1", "%[j3]"),                        \
                  "v_perm_b32 %[pa], %[pa], %[j4], %[ska]\n\t",                              \
                  "v_perm_b32 %[pb], %[pb], %[j4], %[skb]\n\t", "", "")                      \
        "v_lshlrev_b32_e32 %[h1], 16, %[h1]\n\t"                                              \
        "s_setprio 0\n\t"                                                                    \
        "s_branch 3b\n"                                                                      \
        "4:\n\t"                                                                             \
        PC_CNT(3)                                                                            \
        PC_MASKED(PC_RESET("%[h1]", "%[r0]") PC_MCELL("%[c0]", "%[h1]", "a", "WORD_0", "%[j0]"), \
                  PC_RESET("%[c0]", "%[j1]") PC_MCELL("%[c1]", "%[c0]", "a", "WORD_1", "%[j1]"), \
                  PC_RESET("%[c1]", "%[j2]") PC_MCELL("%[c2]", "%[c1]", "b", "WORD_0", "%[j2]"), \
                  PC_RESET("%[c2]", "%[j3]") PC_MCELL("%[h1]", "%[c2]", "b", "WORD_1", "%[j3]"), \
                  "v_perm_b32 %[pa], %[pa], %[j4], %[ska]\n\t",                              \
                  "v_perm_b32 %[pb], %[pb], %[j4], %[skb]\n\t",                              \
                  PC_LEFTMASK("a"), PC_LEFTMASK("b"))                                        \
        "v_lshlrev_b32_e32 %[h1], 16, %[h1]\n\t"                                              \
        "s_setprio 0\n\t"                                                                    \
        "s_branch 3b\n"                                                                      \
        ".subsection 0\n"                                                                    \
        : [ha] "+v"(ha), [hb] "+v"(hb), [ea] "+v"(ea), [eb] "+v"(eb), [f] "+v"(f),           \
          [h1] "+v"(h1), [key] "+v"(key), [y] "=&v"(y), [sa] "=&v"(sa), [sb] "=&v"(sb),     \
          [ta] "=&v"(ta), [tb] "=&v"(tb), [xa] "=&v"(xa), [xb] "=&v"(xb), [c0] "=&v"(c0),    \
          [c1] "=&v"(c1), [c2] "=&v"(c2), [pa] "=&v"(pa), [pb] "=&v"(pb), [fp] "=&v"(fp),   \
          [jja] "=&s"(tja), [jjb] "=&s"(tjb)                                                 \
          PC_CNT_OPS                                                                         \
        : [q] "v"(q), [plo] "v"(plo), [phi] "v"(phi), [oe2] "s"(oe2), [ed2] "s"(ed2),        \
          [ed] "s"(ed), [e0e] "s"(e0e), [ee2] "s"(ee2), [men] "s"(r.enter), [mfa] "s"(r.fast), [mle] "s"(r.left),           \
          [endw] "v"(endw), [endm1w] "v"(endm1w),                                            \
          [begm2w] "v"(begm2w), [endv] "v"(endv), [begv] "v"(begv), [g] "i"(G),             \
          [j4] "s"(J4), [ska] "v"(bs.ka), [skb] "v"(bs.kb), [ija] "i"(JJA), [ijb] "i"(JJB),  \
          [j0] "i"(4 * G), [j1] "i"(4 * G + 1),                                              \
          [j2] "i"(4 * G + 2), [j3] "i"(4 * G + 3), [r0] "i"(R0)                             \
        : "vcc", "scc")

struct PcbSel { uint32_t ka, kb; };            // key selectors (VGPRs: v_perm takes one SGPR)

// One 4-column group G (columns / slots 4G .. 4G+3) as ONE asm statement: skip / FAST /
// MASKED (R: right edge only; L: also resets at beg) decided by scalar tests inside.
template <int G, bool JK>
__device__ __forceinline__ void pc_group(uint32_t &ha, uint32_t &hb, uint32_t &ea, uint32_t &eb,
                                         uint32_t q, uint32_t plo, uint32_t phi, int &f, int &h1,
                                         uint32_t &key, uint32_t oe2, uint32_t ed2, int ed,
                                         const PcRow &r, uint32_t endw, uint32_t endm1w,
                                         uint32_t begm2w, int endv, int begv, const PcbSel &bs,
                                         uint32_t (&ctr)[4])
{
    (void)ctr;
    (void)bs;
    // key slot s carries column j = s - 1: jj = {4G-1, 4G} and {4G+1, 4G+2}
    constexpr uint32_t JJA = ((uint32_t)(4 * G - 1) & 0xffffu) | ((uint32_t)(4 * G) << 16);
    constexpr uint32_t JJB = (uint32_t)(4 * G + 1) | ((uint32_t)(4 * G + 2) << 16);
    constexpr int R0 = (G == 0) ? -1 : 4 * G;   // no reset entering column 0 (the boundary)
    uint32_t y, sa, sb, ta, tb, xa, xb, c0, c1, c2, pa, pb, fp;
    const uint32_t e0e = (uint32_t)ed << 16;                          // {0, e}
    const uint32_t ee2 = (uint32_t)ed | ((uint32_t)(2 * ed) << 16);   // {e, 2e}
    if constexpr (G == 0) {
        // slot 0 holds the column-0 boundary, not a cell: its key half is 0 (c0 << 24 | 0)
        PC_GROUP_ASM("v_lshlrev_b32_e32 %[pa], 24, %[pa]\n\t",        /* pa = {H(0), H(1)} here */
                     "v_lshl_or_b32 %[pa], %[c0], 24, 0\n\t");
    } else if constexpr (JK) {
        constexpr uint32_t J4 = (uint32_t)(4 * G - 1) | ((uint32_t)(4 * G) << 8) | ((uint32_t)(4 * G + 1) << 16) |
                                ((uint32_t)(4 * G + 2) << 24);
        uint32_t tja, tjb;
        PC_GROUP_ASM_J;
    } else {
        PC_GROUP_ASM("v_lshl_or_b32 %[pa], %[ha], 8, %[jja]\n\t",
                     "v_lshl_or_b32 %[pa], %[pa], 8, %[jja]\n\t");
    }
}

// ---- byte planes (BY kernels, BSW_OPT_KERNEL8 = 2): the 8-bit regime's cells stored as bytes
//   HB[G] = bytes {H(i-1, 4G-1), H(i-1, 4G), H(i-1, 4G+1), H(i-1, 4G+2)}   (slots 4G .. 4G+3)
//   EB[G] = bytes {E(i, 4G), .., E(i, 4G+3)}
// half the plane registers of the int16 form.  A group unpacks its two bytes words into the
// int16 pairs the shared arithmetic runs on (4 v_perm, after the skip test: skipped groups pay
// nothing), and packs back: H by the two v_perm that replace the FAST chain's byte-aligns, E by
// one v_perm; the row-max key is built from HB by one v_perm per pair of slots (as v_lshl_or
// before).  Every stored H, E is in [0, 255] (H <= h0 + min(qlen, tlen) <= 255, the planner's
// contract; E <= H and E' clamped at 0 by PC_PH1B).
constexpr uint32_t kSelLo = 0x0C010C00u;       // {b0, b1} of a bytes word -> two int16 halves
constexpr uint32_t kSelHi = 0x0C030C02u;       // {b2, b3}
constexpr uint32_t kSelPk = 0x06040200u;       // v_perm(hi, lo): {lo.w0, lo.w1, hi.w0, hi.w1} -> bytes
constexpr uint32_t kSelA1 = 0x0C060402u;       // v_perm(pa, h1 in): {h1.b2, pa.b0, pa.b2, 0}
constexpr uint32_t kSelA2 = 0x04020100u;       // v_perm(h1 out, t): {t.b0, t.b1, t.b2, h1.b0}
constexpr uint32_t kSelKa = 0x05020400u;       // v_perm(HB, jj): {jj.b0, HB.b0, jj.b2, HB.b1} = H << 8 | j
constexpr uint32_t kSelKb = 0x07020600u;       // {jj.b0, HB.b2, jj.b2, HB.b3}
constexpr uint32_t kSelK0 = 0x050C0C0Cu;       // group 0: {0, 0, 0, HB.b1} (slot 0 is no cell)

#define PCB_UNPACK                                                                       \
    "v_perm_b32 %[ha], %[hw], %[hw], %[slo]\n\t"                                             \
    "v_perm_b32 %[hb], %[hw], %[hw], %[shi]\n\t"                                             \
    "v_perm_b32 %[ea], %[ew], %[ew], %[slo]\n\t"                                             \
    "v_perm_b32 %[eb], %[ew], %[ew], %[shi]\n\t"
#define PCB_PACK                                                                         \
    "v_perm_b32 %[hw], %[hb], %[ha], %[spk]\n\t"                                             \
    "v_perm_b32 %[ew], %[eb], %[ea], %[spk]\n\t"

#define PCB_GROUP_ASM(KEYA_FAST, KEYA_MASK)                                               \
    asm volatile(                                                                            \
        "s_bitcmp1_b64 %[mfa], %[g]\n\t"             /* every live lane in band: FAST */    \
        "s_cbranch_scc0 5f\n\t"                                                              \
        PC_CNT(0) PC_CNT(1)                                                                  \
        PCB_UNPACK                                                                           \
        PC_SCORES                                                                            \
        PC_PH1B("a", "%[ea]") PC_PH1B("b", "%[eb]")                                          \
        PC_FAST_CHAIN_("v_perm_b32 %[hw], %[pa], %[h1], %[sa1]\n\t",                         \
                       "v_perm_b32 %[hw], %[h1], %[hw], %[sa2]\n\t")                         \
        "v_perm_b32 %[ew], %[eb], %[ea], %[spk]\n\t"                                         \
        KEYA_FAST                                                                            \
        "v_pk_max_u16 %[key], %[key], %[pa]\n\t"                                             \
        "v_perm_b32 %[pb], %[hw], %[jjb], %[vkb]\n\t"                                        \
        "v_pk_max_u16 %[key], %[key], %[pb]\n"                                               \
        "3:\n"                                                                               \
        ".subsection 1\n"                                                                    \
        "5:\n\t"                                                                             \
        "s_bitcmp1_b64 %[men], %[g]\n\t"             /* outside [min beg, max end]: skip */ \
        "s_cbranch_scc0 3b\n\t"                                                              \
        "s_setprio 2\n\t"                                                                    \
        PC_CNT(0)                                                                            \
        PCB_UNPACK                                                                           \
        "v_lshrrev_b32_e32 %[h1], 16, %[h1]\n\t"                                             \
        PC_SCORES                                                                            \
        "s_bitcmp1_b64 %[mle], %[g]\n\t"             /* some lane's beg in this group: L */ \
        "s_cbranch_scc1 4f\n\t"                                                              \
        PC_CNT(2)                                                                            \
        PC_MASKED_(PC_PH1B,                                                                  \
                  PC_MCELL("%[c0]", "%[h1]", "a", "WORD_0", "%[j0]"),                        \
                  PC_MCELL("%[c1]", "%[c0]", "a", "WORD_1", "%[j1]"),                        \
                  PC_MCELL("%[c2]", "%[c1]", "b", "WORD_0", "%[j2]"),                        \
                  PC_MCELL("%[h1]", "%[c2]", "b", "WORD_1", "%[j3]"),                        \
                  KEYA_MASK, "v_lshl_or_b32 %[pb], %[pb], 8, %[jjb]\n\t", "", "")           \
        PCB_PACK                                                                             \
        "v_lshlrev_b32_e32 %[h1], 16, %[h1]\n\t"                                             \
        "s_setprio 0\n\t"                                                                    \
        "s_branch 3b\n"                                                                      \
        "4:\n\t"                                                                             \
        PC_CNT(3)                                                                            \
        PC_MASKED_(PC_PH1B,                                                                  \
                  PC_RESET("%[h1]", "%[r0]") PC_MCELL("%[c0]", "%[h1]", "a", "WORD_0", "%[j0]"), \
                  PC_RESET("%[c0]", "%[j1]") PC_MCELL("%[c1]", "%[c0]", "a", "WORD_1", "%[j1]"), \
                  PC_RESET("%[c1]", "%[j2]") PC_MCELL("%[c2]", "%[c1]", "b", "WORD_0", "%[j2]"), \
                  PC_RESET("%[c2]", "%[j3]") PC_MCELL("%[h1]", "%[c2]", "b", "WORD_1", "%[j3]"), \
                  KEYA_MASK, "v_lshl_or_b32 %[pb], %[pb], 8, %[jjb]\n\t",                    \
                  PC_LEFTMASK("a"), PC_LEFTMASK("b"))                                        \
        PCB_PACK                                                                             \
        "v_lshlrev_b32_e32 %[h1], 16, %[h1]\n\t"                                             \
        "s_setprio 0\n\t"                                                                    \
        "s_branch 3b\n"                                                                      \
        ".subsection 0\n"                                                                    \
        : [hw] "+v"(hw), [ew] "+v"(ew), [ha] "=&v"(ha), [hb] "=&v"(hb), [ea] "=&v"(ea),      \
          [eb] "=&v"(eb), [f] "+v"(f),                                                       \
          [h1] "+v"(h1), [key] "+v"(key), [y] "=&v"(y), [sa] "=&v"(sa), [sb] "=&v"(sb),     \
          [ta] "=&v"(ta), [tb] "=&v"(tb), [xa] "=&v"(xa), [xb] "=&v"(xb), [c0] "=&v"(c0),    \
          [c1] "=&v"(c1), [c2] "=&v"(c2), [pa] "=&v"(pa), [pb] "=&v"(pb), [fp] "=&v"(fp)    \
          PC_CNT_OPS                                                                         \
        : [q] "v"(q), [plo] "v"(plo), [phi] "v"(phi), [oe2] "s"(oe2), [ed2] "s"(ed2),        \
          [ed] "s"(ed), [e0e] "s"(e0e), [ee2] "s"(ee2), [men] "s"(r.enter), [mfa] "s"(r.fast), [mle] "s"(r.left),           \
          [endw] "v"(endw), [endm1w] "v"(endm1w),                                            \
          [begm2w] "v"(begm2w), [endv] "v"(endv), [begv] "v"(begv), [g] "i"(G),             \
          [jja] "s"(JJA), [jjb] "s"(JJB), [j0] "i"(4 * G), [j1] "i"(4 * G + 1),              \
          [j2] "i"(4 * G + 2), [j3] "i"(4 * G + 3), [r0] "i"(R0),                            \
          [slo] "s"(kSelLo), [shi] "s"(kSelHi), [spk] "s"(kSelPk), [sa1] "s"(kSelA1),         \
          [sa2] "s"(kSelA2), [sk0] "s"(kSelK0), [vka] "v"(bs.ka), [vkb] "v"(bs.kb)            \
        : "vcc", "scc")


template <int G>
__device__ __forceinline__ void pcb_group(uint32_t &hw, uint32_t &ew, uint32_t q, uint32_t plo, uint32_t phi,
                                          int &f, int &h1, uint32_t &key, uint32_t oe2, uint32_t ed2, int ed,
                                          const PcRow &r, uint32_t endw, uint32_t endm1w, uint32_t begm2w,
                                          int endv, int begv, const PcbSel &bs, uint32_t (&ctr)[4])
{
    (void)ctr;
    constexpr uint32_t JJA = ((uint32_t)(4 * G - 1) & 0xffffu) | ((uint32_t)(4 * G) << 16);
    constexpr uint32_t JJB = (uint32_t)(4 * G + 1) | ((uint32_t)(4 * G + 2) << 16);
    constexpr int R0 = (G == 0) ? -1 : 4 * G;
    uint32_t ha, hb, ea, eb, y, sa, sb, ta, tb, xa, xb, c0, c1, c2, pa, pb, fp;
    const uint32_t e0e = (uint32_t)ed << 16;
    const uint32_t ee2 = (uint32_t)ed | ((uint32_t)(2 * ed) << 16);
    if constexpr (G == 0) {
        PCB_GROUP_ASM("v_perm_b32 %[pa], %[hw], %[hw], %[sk0]\n\t",
                      "v_lshl_or_b32 %[pa], %[c0], 24, 0\n\t");
    } else {
        PCB_GROUP_ASM("v_perm_b32 %[pa], %[hw], %[jja], %[vka]\n\t",
                      "v_lshl_or_b32 %[pa], %[pa], 8, %[jja]\n\t");
    }
}

// plane registers per pair: two columns per VGPR (int16), four (bytes)
template <int QMAX, bool BY> struct PcNp { static constexpr int v = BY ? QMAX / 4 : QMAX / 2; };

template <int QMAX, bool BY, int G>
__device__ __forceinline__ void pc_group_if(uint32_t (&hh)[(BY ? QMAX / 4 : QMAX / 2)], uint32_t (&ee)[(BY ? QMAX / 4 : QMAX / 2)],
                                            const uint32_t (&qs)[QMAX / 4], uint32_t plo, uint32_t phi, int &f,
                                            int &h1, uint32_t &key, uint32_t oe2, uint32_t ed2, int ed,
                                            const PcRow &r, uint32_t endw, uint32_t endm1w, uint32_t begm2w, int endv,
                                            int begv, const PcbSel &bs, uint32_t (&ctr)[4])
{
    if constexpr (G < QMAX / 4) {
        if constexpr (BY)
            pcb_group<G>(hh[G], ee[G], qs[G], plo, phi, f, h1, key, oe2, ed2, ed, r, endw, endm1w, begm2w, endv,
                         begv, bs, ctr);
        else
            pc_group<G, BSW_PC_JKEY && QMAX >= 128>(hh[2 * G], hh[2 * G + 1], ee[2 * G], ee[2 * G + 1], qs[G], plo, phi, f, h1, key, oe2, ed2,
                        ed, r, endw, endm1w, begm2w, endv, begv, bs, ctr);
    }
}

// Segments of 8 groups behind one uniform test of the row's entered set: a segment no lane's
// band touches costs one s_and + branch instead of 8 x (FAST test + skip test + 2 branches)
// (one segment, no test, for QMAX <= 64: the tests' registers would cost the 64 class its
// fourth wave per SIMD, 127 -> 137 VGPRs)
#ifndef BSW_PC_SEG             // experiment builds (make ab AB_FLAGS=-DBSW_PC_SEG=4) only
#define BSW_PC_SEG 8
#endif
constexpr int kPcSeg = BSW_PC_SEG;
template <int QMAX> constexpr int pc_seg_len() { return QMAX <= 64 ? QMAX / 4 : kPcSeg; }
template <int QMAX, bool BY, int S, int... K>
__device__ __forceinline__ void pc_seg(std::integer_sequence<int, K...>, uint32_t (&hh)[(BY ? QMAX / 4 : QMAX / 2)],
                                       uint32_t (&ee)[(BY ? QMAX / 4 : QMAX / 2)], const uint32_t (&qs)[QMAX / 4], uint32_t plo,
                                       uint32_t phi, int &f, int &h1, uint32_t &key, uint32_t oe2, uint32_t ed2,
                                       int ed, const PcRow &r, uint32_t endw, uint32_t endm1w, uint32_t begm2w,
                                       int endv, int begv, const PcbSel &bs, uint32_t (&ctr)[4])
{
    constexpr int kSeg = sizeof...(K);
    constexpr uint64_t kSegMask = ((1ull << kSeg) - 1) << (kSeg * S);
    if (kSeg == QMAX / 4 || (r.enter & kSegMask))
        (pc_group_if<QMAX, BY, kSeg * S + K>(hh, ee, qs, plo, phi, f, h1, key, oe2, ed2, ed, r, endw, endm1w,
                                               begm2w, endv, begv, bs, ctr), ...);
}

template <int QMAX, bool BY, int... S>
__device__ __forceinline__ void pc_row(std::integer_sequence<int, S...>, uint32_t (&hh)[(BY ? QMAX / 4 : QMAX / 2)],
                                       uint32_t (&ee)[(BY ? QMAX / 4 : QMAX / 2)], const uint32_t (&qs)[QMAX / 4],
                                       uint32_t plo, uint32_t phi, int &f, int &h1, uint32_t &key,
                                       uint32_t oe2, uint32_t ed2, int ed, const PcRow &r,
                                       uint32_t endw, uint32_t endm1w, uint32_t begm2w, int endv,
                                       int begv, const PcbSel &bs, uint32_t (&ctr)[4])
{
    (pc_seg<QMAX, BY, S>(std::make_integer_sequence<int, pc_seg_len<QMAX>()>{}, hh, ee, qs, plo, phi, f, h1, key, oe2,
                         ed2, ed, r, endw, endm1w, begm2w, endv, begv, bs, ctr), ...);
}

// Lazy last positive column: when H(i, end-1) == 0 the lanes that need it
// look for the last slot s <= end (slot s = H(i, s-1)) holding H > 0; lp1 = that slot = 1 + lastH.
// Packed scan, two slots per instruction, registers from the one holding slot max(end) down:
//   c = min(H, 1) * s (slot or 0), cleared where s > end, lp = max(lp, c)
// 6 packed ops per register; a uniform test after each pair of registers stops the scan once
// every needing lane found its slot.  Slot 0 (the column -1 boundary) contributes 0 = none.
template <int K>
__device__ __forceinline__ void pc_lastpos_reg(uint32_t hv, uint32_t endp1w, uint32_t &lp)
{
    constexpr uint32_t SC = (uint32_t)(2 * K) | ((uint32_t)(2 * K + 1) << 16);
    uint32_t c, m;
    asm volatile(
        "v_pk_min_u16 %[c], %[h], 1 op_sel_hi:[1,0]\n\t"
        "v_pk_mul_lo_u16 %[c], %[c], %[sc]\n\t"
        "v_pk_sub_i16 %[m], %[sc], %[e1]\n\t"               // s - (end + 1) < 0  <=>  s <= end
        "v_pk_ashrrev_i16 %[m], 15, %[m] op_sel_hi:[0,1]\n\t"
        "v_and_b32_e32 %[c], %[c], %[m]\n\t"
        "v_pk_max_u16 %[lp], %[lp], %[c]\n\t"
        : [lp] "+v"(lp), [c] "=&v"(c), [m] "=&v"(m)
        : [h] "v"(hv), [sc] "s"(SC), [e1] "v"(endp1w));
}

template <int QMAX, bool BY, int GG>
__device__ __forceinline__ bool pc_lastpos_group(const uint32_t (&hh)[(BY ? QMAX / 4 : QMAX / 2)], uint32_t endp1w,
                                                 bool pending, uint32_t &lp, int gstart)
{
    if (GG > gstart) return pending;                      // uniform: above every lane's end
    if (__ballot(pending) == 0) return false;             // uniform: all found
    if constexpr (BY) {                                   // slots {4GG+2, 4GG+3}, {4GG, 4GG+1}
        pc_lastpos_reg<2 * GG + 1>(__builtin_amdgcn_perm(hh[GG], hh[GG], kSelHi), endp1w, lp);
        pc_lastpos_reg<2 * GG>(__builtin_amdgcn_perm(hh[GG], hh[GG], kSelLo), endp1w, lp);
    } else {
        if constexpr (2 * GG + 1 < QMAX / 2) pc_lastpos_reg<2 * GG + 1>(hh[2 * GG + 1], endp1w, lp);
        pc_lastpos_reg<2 * GG>(hh[2 * GG], endp1w, lp);
    }
    return pending & (lp == 0u);
}

template <int QMAX, bool BY, int... G>
__device__ __forceinline__ int pc_lastpos(std::integer_sequence<int, G...>, const uint32_t (&hh)[(BY ? QMAX / 4 : QMAX / 2)],
                                          int end, bool need, int gstart)
{
    bool pending = need;
    uint32_t lp = 0;
    const uint32_t endp1w = pack2(end + 1);
    ((pending = pc_lastpos_group<QMAX, BY, QMAX / 4 - 1 - G>(hh, endp1w, pending, lp, gstart)), ...);
    return (int)max(lp & 0xffffu, lp >> 16);
}

// WPB waves per workgroup: with 1, a wave's slot (and its LDS) is reused as soon as that wave
// ends, instead of when the slowest of its block's waves ends.
template <int QMAX, int WPB, bool BY>
__global__ __launch_bounds__(64 * WPB, BY ? 3 : 2) void pc_kernel(const KParams kp, const int32_t w,
                                                    SeqPair *__restrict__ pairs,
                                                    const int32_t *__restrict__ order,
                                                    const int32_t n,
                                                    const uint8_t *__restrict__ ref,
                                                    const uint8_t *__restrict__ qer,
                                                    int32_t *__restrict__ err)
{
    constexpr int NG = QMAX / 4;        // groups = query words (4 codes each)
    constexpr int CDW = kPcChunkDw;     // target dwords per lane per 64-row chunk
#ifdef BSW_PC_STATS
    const unsigned long long t_wave0 = wall_clock64();
#endif
    __shared__ uint32_t s_tgt[WPB][2][CDW][64];   // 8.7 KB per wave
    __shared__ uint2 s_prof[8];                           // per-row score profiles, by target code
    if (threadIdx.x < 8) s_prof[threadIdx.x] = make_uint2(kp.prof[threadIdx.x][0], kp.prof[threadIdx.x][1]);
    __syncthreads();
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = gid < n;
    const int idx = valid ? (order ? order[gid] : gid) : 0;
    SeqPair *sp = pairs + idx;
    int idr = 0, idq = 0, tlen = 0, qlen = 0, h0 = 0;
    if (valid) {
        idr = sp->idr; idq = sp->idq; tlen = sp->len1; qlen = sp->len2; h0 = sp->h0;
        if (qlen >= QMAX || qlen < 0 || tlen < 0 || h0 < 0 || h0 + min(qlen, tlen) > 255 || idr < 0 || idq < 0) {
            atomicOr(err, 1);
            valid = false;
        }
    }
    // query codes, 4 per VGPR in byte order {c0, c2, c1, c3}: aligned dword loads (a dword
    // holding a byte of the query never leaves that byte's page), realigned by v_alignbyte
    uint32_t qs[NG];
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
        for (int g = 0; g < NG; ++g) {
            const uint32_t c = __builtin_amdgcn_alignbyte(wv[g + 1], wv[g], sh);
            qs[g] = __builtin_amdgcn_perm(c, c, 0x03010200u);
        }
    }
    // A.1 first row: slot 0 = h0, slot j = max(h0 - oe_ins - (j-1) e_ins, 0) for 1 <= j <= qlen
    constexpr int NP = (BY ? QMAX / 4 : QMAX / 2);
    uint32_t hh[NP], ee[NP];
    {
        const int oe_ins = kp.o_ins + kp.e_ins;
        if constexpr (BY) {
            __builtin_amdgcn_sched_barrier(0);     // after the query words: their loads' registers
                                                   // are dead before the planes are built
#pragma unroll
            for (int k = 0; k < NP; ++k) {         // h0 <= 255 (the 8-bit regime): bytes
                uint32_t v[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int j = 4 * k + t;
                    v[t] = (j == 0) ? (uint32_t)h0 : (j <= qlen) ? (uint32_t)max(h0 - oe_ins - (j - 1) * kp.e_ins, 0) : 0u;
                }
                hh[k] = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
                asm volatile("" : "+v"(hh[k]));   // built here, not sunk to the loop (the
                ee[k] = 0u;                        // bytes of every word live at once: +40 VGPRs)
            }
        } else {
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                const int j0 = 2 * k, j1 = 2 * k + 1;
                const uint32_t a = (j0 == 0) ? (uint32_t)h0
                                 : (j0 <= qlen) ? (uint32_t)max(h0 - oe_ins - (j0 - 1) * kp.e_ins, 0) : 0u;
                const uint32_t b = (j1 <= qlen) ? (uint32_t)max(h0 - oe_ins - (j1 - 1) * kp.e_ins, 0) : 0u;
                hh[k] = a | (b << 16);
                ee[k] = 0u;
            }
        }
    }
    // A.2 per-lane band cap, integer form of (int)((double)N / e + 1.)
    int wl = w;
    {
        const int ni = qlen * kp.maxsc + kp.end_bonus - kp.o_ins;
        const int nd = qlen * kp.maxsc + kp.end_bonus - kp.o_del;
        wl = min(wl, max((ni + kp.e_ins) / kp.e_ins, 1));
        wl = min(wl, max((nd + kp.e_del) / kp.e_del, 1));
    }
    int best = h0, best_i = -1, best_j = -1, max_ie = -1, gsc = -1, moff = 0, endc = qlen;
    bool alive = valid && tlen > 0;
    // target bases HBM -> LDS by LDS-DMA, 64-row chunks double-buffered (as the lane kernel)
    const uint8_t *tp = ref + idr;
    const int tsh = (int)((uintptr_t)tp & 3);
    const uint32_t *twp = (const uint32_t *)(tp - tsh);
    const int tlast = max((tsh + tlen - 1) >> 2, 0);
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    auto issue_chunk = [&](int ch) {
        uint32_t *dst = &s_tgt[wv][ch & 1][0][0];
#pragma unroll
        for (int k = 0; k < CDW; ++k)
            __builtin_amdgcn_global_load_lds((gptr_t)(twp + min(16 * ch + k, tlast)),
                                             (lptr_t)(dst + 64 * k), 4, 0, 0);
    };
    if (alive) { issue_chunk(0); issue_chunk(1); }
    uint32_t tcur = 0;
    const int wl_max = wave_max(alive ? wl : -1);
    const int wl_min = wave_min(alive ? wl : INT_MAX);
    const uint32_t oe2 = (uint32_t)(kp.o_del + kp.e_del) * 0x10001u;
    const uint32_t ed2 = (uint32_t)kp.e_del * 0x10001u;
    uint32_t ctr[4] = {0, 0, 0, 0};                       // BSW_PC_STATS group-path counters
    // key selectors in VGPRs: the byte planes' (BY) or the JKEY ones (int16 planes)
    // (the JKEY selectors only where the two VGPRs cost no occupancy: QMAX >= 128 runs at two
    // waves per SIMD either way; the 96 / 64 classes would drop from 3 / 4 waves)
    PcbSel bs{BY ? kSelKa : 0x06010400u, BY ? kSelKb : 0x06030402u};
    if constexpr (BY || (BSW_PC_JKEY && QMAX >= 128)) asm volatile("" : "+v"(bs.ka), "+v"(bs.kb));
#ifdef BSW_PC_STATS
    uint32_t nrows = 0, nlast = 0, nue = 0;
#endif

#if BSW_PC_EXP_HALFHEAD
    int emax = 0, emin = 0;                 // (experiment: the row head's state outlives its row)
    PcRow r{0, 0, 0};
#endif
    for (int i = 0;; ++i) {
        const bool act = alive && i < tlen;
        alive = act;
        if (__ballot(act) == 0) break;
        // the row's target base and score profile first: their LDS reads then overlap the band
        // bookkeeping below instead of stalling the first group (lgkmcnt wait)
        // every lane reads (a dead lane's slots are harmless): no exec-masked block on the row's path
        if ((i & 3) == 0) {                // new 4-row block: bases from LDS
            if ((i & 63) == 0) {              // chunk boundary: its DMA was issued 64 rows ago
                __builtin_amdgcn_s_waitcnt(0x0F70);      // vmcnt(0)
                __builtin_amdgcn_sched_barrier(0);
            }
            const int k = (i >> 2) & 15;
            // the two dwords by inline asm: the compiler would otherwise put a vmcnt(0) before
            // every LDS read (it cannot tell this buffer from the one the in-flight LDS-DMA
            // refill writes) -- this chunk's DMA was waited for at its first row above
            const uint32_t la = (uint32_t)(uintptr_t)(lptr_t)&s_tgt[wv][(i >> 6) & 1][k][ln];
            uint2 d;
            asm volatile("ds_read2st64_b32 %0, %1 offset1:1\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(d) : "v"(la) : "memory");
            tcur = __builtin_amdgcn_alignbyte(d.y, d.x, tsh);
            if ((i & 63) == 0) {
                __builtin_amdgcn_sched_barrier(0);
                if (i > 0 && act) issue_chunk((i >> 6) + 1);   // refill the buffer just drained
            }
        }
        // per-row score profile of target base t (8 bytes: mat[t][q], q = 0..7)
        const uint32_t tcode = (tcur >> (8 * (i & 3))) & 0xffu;
        const uint2 pr = s_prof[min(tcode, 7u)];   // one ds_read_b64 (codes > 4 score as N)
        __builtin_amdgcn_sched_barrier(0);
        const int beg = max(0, i - wl);
        const int end = min(min(endc, i + wl + 1), qlen);
        endc = end;
#if BSW_PC_EXP_HALFHEAD
        // experiment build only (make ab AB_FLAGS=-DBSW_PC_EXP_HALFHEAD=1; WRONG outputs): the row
        // head -- band-end reductions and the three group sets -- on even rows only, the odd rows
        // reusing the previous row's: the time a two-rows-per-pass schedule could save on row heads
        // (-1.3%)
        if (i & 1) goto row_body;
#else
        int emax, emin;
        PcRow r;
#endif
        wave_maxmin_bc(act ? end : -1, act ? end : INT_MAX, emax, emin);
        {
            const int ulo = __builtin_amdgcn_readfirstlane(max(0, i - wl_max));  // min beg
            const int uhi = __builtin_amdgcn_readfirstlane(emax);                // max end
            const int flo = __builtin_amdgcn_readfirstlane(max(0, i - wl_min));  // max beg
            const int fhi = __builtin_amdgcn_readfirstlane(emin);                // min end
            const int glo = ulo >> 2;
            const int gsp = max((min(uhi, QMAX - 1) >> 2) - glo, -1);      // uhi >= 0: a live lane
            // FAST needs 4G > every beg (entering chain valid) -- or one common beg == 4G with
            // nothing computed before it -- and 4G + 4 <= every end
            const int gfa = (ulo == flo && (flo & 3) == 0) ? (flo >> 2) : (flo >> 2) + 1;
            const int gfn = max((fhi >> 2) - gfa, 0);
            const int gln = (flo >> 2) - glo;
            r.enter = gbits(glo, gsp + 1);
            r.fast = gbits(gfa, gfn);
            r.left = gbits(glo, gln + 1);
        }
#if BSW_PC_EXP_HALFHEAD
    row_body:
#endif
        {   // every lane runs the row (dead lanes' registers take garbage); state updates are
            // gated by act below, so no exec-masked block wraps the row
            // h1 = H(i, j-1) entering each group, in the HIGH half (PC_FAST_CHAIN)
            // (a mask, not a select: the compiler turned the select into an exec-masked block)
            int h1 = (int)((uint32_t)max(h0 - (kp.o_del + kp.e_del * (i + 1)), 0) << 16) & -(int)(beg == 0);
            int f = 0;
            uint32_t key = 0;
            const uint32_t endw = pack2(end);
            const uint32_t endm1w = pack2(end - 1);                         // end = 0: {-1, -1}
            const uint32_t begm2w = pack2(beg - 2);
            // wave priority: the row's serial scalar / DPP chain (row end, next row's head) issues
            // ahead of the partner wave's group VALU; the groups themselves run at the base level
            __builtin_amdgcn_s_setprio(0);
            pc_row<QMAX, BY>(std::make_integer_sequence<int, (NG + pc_seg_len<QMAX>() - 1) / pc_seg_len<QMAX>()>{}, hh, ee,
                             qs, pr.x, pr.y, f, h1, key, oe2, ed2, kp.e_del, r, endw, endm1w, begm2w, end, beg, bs,
                             ctr);
            __builtin_amdgcn_s_setprio(2);
            h1 = (int)((uint32_t)h1 >> 16);               // H(i, end-1)
            const uint32_t k32 = max(key & 0xffffu, key >> 16);
            const int m = (int)(k32 >> 8), mj = (int)(k32 & 0xffu);
            {                                     // A.4: j == qlen; h1 = H(i, qlen - 1)
                const bool atq = act && end == qlen;
                max_ie = (atq && !(gsc > h1)) ? i : max_ie;
                gsc = atq ? max(gsc, h1) : gsc;
            }
            // A.4 row end as selects, no branches on the row's path: m <= 0 ends the lane; a new
            // best moves (best, best_i, best_j, max_off); otherwise z-drop against the old best
            {
                const int di = i - best_i, dj = mj - best_j;
                // |di - dj| and e are small and non-negative: 24-bit multiplies (full rate)
                const int dz = (di > dj) ? best - m - (int)__umul24((unsigned)(di - dj), (unsigned)kp.e_del)
                                         : best - m - (int)__umul24((unsigned)(dj - di), (unsigned)kp.e_ins);
                const bool better = act && m > best;       // best >= h0 >= 0: never with m <= 0
                const bool zdropped = kp.zdrop > 0 && dz > kp.zdrop;
                alive = act && m > 0 && (better || !zdropped);
                moff = better ? max(moff, abs(mj - i)) : moff;
                best_i = better ? i : best_i;
                best_j = better ? mj : best_j;
                best = better ? m : best;
            }
#ifdef BSW_PC_STATS
            nrows += act;
            nue += act && (emax == emin);  // every live lane has the same band end
#endif
            {                                      // end_{i+1} = min(lastH + 3, ...), DESIGN.md §3
                const bool need = alive && h1 == 0;  // H(i, end-1) == 0 -> lastH < end - 1
                int lp1 = end;
                if (__ballot(need)) {
#ifdef BSW_PC_STATS
                    nlast += 1;
#endif
                    const int lp = pc_lastpos<QMAX, BY>(std::make_integer_sequence<int, NG>{}, hh, end, need,
                                                        emax >> 2);
                    lp1 = need ? lp : end;
                }
                endc = alive ? min(lp1 + 2, qlen) : endc;
            }
        }
    }
#ifdef BSW_PC_STATS
    {   // per wave: rows (max over lanes), group paths, lastpos scans; lane 0 adds
        const unsigned rows = (unsigned)wave_max((int)nrows);
        const unsigned nl = (unsigned)wave_max((int)nlast);
        const unsigned nu = (unsigned)wave_max((int)nue);
        unsigned cmax[4];
        for (int k = 0; k < 4; ++k) cmax[k] = (unsigned)wave_max((int)ctr[k]);   // the longest lane
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&g_pc_stats[0], (unsigned long long)rows);
            for (int k = 0; k < 4; ++k) atomicAdd(&g_pc_stats[1 + k], (unsigned long long)cmax[k]);
            atomicAdd(&g_pc_stats[5], (unsigned long long)nl);
            atomicAdd(&g_pc_stats[6], 1ull);
            atomicAdd(&g_pc_stats[7], (unsigned long long)nu);
        }
        const unsigned wid = blockIdx.x * WPB + (threadIdx.x >> 6);
        if ((threadIdx.x & 63) == 0 && wid < (unsigned)kPcTimesMax) {
            unsigned xcc, hw;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            g_pc_times[wid][0] = t_wave0;
            g_pc_times[wid][1] = wall_clock64();
            g_pc_times[wid][2] = ((unsigned long long)xcc << 32) | hw;
            g_pc_times[wid][3] = rows;
        }
    }
#endif
    if (valid) {
        sp->score = best;
        sp->tle = best_i + 1;
        sp->gtle = max_ie + 1;
        sp->qle = best_j + 1;
        sp->gscore = gsc;
        sp->max_off = moff;
    }
}

#ifdef BSW_PC_STATS
// [rows, groups entered, fast, masked-R, masked-L, lastpos scans, waves, uniform-end rows] summed over waves
extern "C" int bsw_pc_stats(unsigned long long *out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pc_stats), 8 * sizeof(unsigned long long)) != hipSuccess) return -5;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pc_stats), z, sizeof(z)) != hipSuccess) return -5;
    }
    return 0;
}
// the per-wave schedule records of the last launch (n waves, 4 x u64 each)
extern "C" int bsw_pc_times(unsigned long long *out, int n)
{
    n = n < kPcTimesMax ? n : kPcTimesMax;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pc_times), (size_t)n * 32) != hipSuccess) return -5;
    return n;
}
#endif

template <int QMAX>
static void launch_pc_q(const KParams &kp, int32_t w, SeqPair *pairs, const int32_t *order, int32_t n,
                        const uint8_t *ref, const uint8_t *qer, int32_t *err, hipStream_t s)
{
    const unsigned grid = (unsigned)((n + 63) / 64);
    // one wave per workgroup: a finished wave's slot and LDS are reused at once
    if (kp.kern8 == 2)                 // byte planes (BSW_OPT_KERNEL8 = 2)
        hipLaunchKernelGGL((pc_kernel<QMAX, 1, true>), dim3(grid), dim3(64), 0, s, kp, w, pairs, order, n,
                           ref, qer, err);
    else
        hipLaunchKernelGGL((pc_kernel<QMAX, 1, false>), dim3(grid), dim3(64), 0, s, kp, w, pairs, order,
                           n, ref, qer, err);
}

hipError_t launch_pc_kernel(int qmax, const KParams &kp, int32_t w, SeqPair *pairs,
                            const int32_t *order, int32_t n, const uint8_t *ref,
                            const uint8_t *qer, int32_t *err, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    switch (qmax) {
    case 32: launch_pc_q<32>(kp, w, pairs, order, n, ref, qer, err, s); break;
    case 64: launch_pc_q<64>(kp, w, pairs, order, n, ref, qer, err, s); break;
    case 96: launch_pc_q<96>(kp, w, pairs, order, n, ref, qer, err, s); break;
    case 128: launch_pc_q<128>(kp, w, pairs, order, n, ref, qer, err, s); break;
    case 160: launch_pc_q<160>(kp, w, pairs, order, n, ref, qer, err, s); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace bsw
