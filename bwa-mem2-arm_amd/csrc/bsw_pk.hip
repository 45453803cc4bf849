// bsw_pk.hip -- the packed "two pairs per lane" seed-extension kernel for gfx950
// (DESIGN.md §4.2).  Same ksw_extend2 semantics as the lane kernel (SURVEY.md Appendix A,
// exact reformulations DESIGN.md §3); different mapping onto CDNA4:
//
//   Measured on MI355X (tools/valu_issue_bench*.hip): a SIMD issues one
//   ordinary VALU instruction every ~4.5 cycles for everything this recurrence needs (32-bit
//   max/min, SDWA, VOP3, v_perm, compares) no matter how many waves it holds, and a packed
//   16-bit VOP3P instruction (v_pk_max_i16, v_pk_add_u16, ...) costs the same ~4.6 cycles
//   while doing two lanes' worth of work.  So the kernel packs TWO SeqPairs into every lane:
//   pair A in the low 16 bits and pair B in the high 16 bits of each DP register, and every
//   step of the recurrence is a v_pk_* instruction (2 cells per issue slot).
//
//   Per lane (wave = 128 pairs):  HH[j] = {H_A(i-1,j-1), H_B(i-1,j-1)} in arch VGPRs,
//   EE[j] = {E_A(i,j), E_B(i,j)} and the query codes QP[k] (2 columns x 2 pairs) in AGPRs
//   (VALU operands can only name v0..v255: E moves through v_accvgpr_read/write, 2 per
//   column, QP 2 reads per group).  ~500 registers: one wave per SIMD.
//
//   Scores without a per-row profile: S = v_perm(TAB, C ^ T) where C = the column's query
//   codes (duplicated per byte pair), T = the row's target encoding (per pair) and TAB = 8
//   constant bytes {a, -b, -b, -b, -1, -1, -1, -1}; the XOR lands every (query, target) code
//   combination on a selector whose low byte picks the score and whose high byte picks its
//   sign (0x00 / 0xFF, or v_perm's sign-replicate selectors 8..11), giving the exact int16
//   score of both pairs in 3 instructions per column.
//
// Eligibility (planner): bwa-style scoring (match 1, mismatch -b, N -1, symmetric gaps),
// h0 + min(qlen, tlen) <= 255 so that key = H << 8 | j fits 16 bits, qlen <= QMAX.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include <utility>
#include "bsw_kernels.h"
#include "bsw_wave.h"

namespace bsw {

constexpr int kPkChunkDw = 17;           // dwords per lane per 64-row target chunk (as lane kernel)

struct PkRow {                           // per-row uniform (SGPR) group bounds
    int glo, gsp;                        // groups touching [min beg, max end]
    int gfa, gfn;                        // groups with every live pair in band
};

struct PkHalf {                          // one pair's scalar state (A = low half, B = high)
    int h0, qlen, tlen, wl;
    int best, best_i, best_j, max_ie, gsc, moff, endc;
    bool valid, alive;
};

// One 4-column group (columns J0 = 4G .. J0+3) of both pairs as ONE asm statement
// (in-place update of HH/EE/f/key, no control-flow merge copies):
//   skip    : group outside [min beg, max end] of the live pairs (scalar test)
//   phase 1 : scores, gated M = hold + min(S, hold), t = max(M - oe, 0), max(M, E), E - e
//   fast    : every live pair in band: F chain, H, E', key = max(H<<8 | j); 8 instr per column
//             (the last positive column is recovered lazily at row end, pk_lastpos)
//   masked  : per-half masks OUT = (j >= end), GT = (j > end), LEFT = (j < beg) from packed
//             arithmetic; stores beyond end preserved (A.7), E' = 0 at j == end, F reset left
//             of beg, masked cells feed 0 to key; hg passes H(i, end-1) along for gscore (only
//             in-band cells update it: an empty row keeps the boundary value).
#ifdef PK_EXP_NO_AGPR
#define PK_ACCR(d, a) "v_mov_b32 " d ", " a "\n\t"
#define PK_ACCW(a, d) "v_mov_b32 " a ", " d "\n\t"
#define PK_ECON "+v"
#define PK_QCON "v"
#else
#define PK_ACCR(d, a) "v_accvgpr_read_b32 " d ", " a "\n\t"
#define PK_ACCW(a, d) "v_accvgpr_write_b32 " a ", " d "\n\t"
#define PK_ECON "+a"
#define PK_QCON "a"
#endif
#ifdef PK_EXP_NO_TESTS
#define PK_TESTS(a, b)
#define PK_SLOW(...)
#else
#define PK_TESTS(a, b) a b
#define PK_SLOW(...) __VA_ARGS__
#endif

template <int G>
__device__ __forceinline__ void pk_group(uint32_t &h0, uint32_t &h1, uint32_t &h2, uint32_t &h3,
                                         uint32_t &e0, uint32_t &e1, uint32_t &e2, uint32_t &e3,
                                         uint32_t hn, uint32_t qa, uint32_t qb, uint32_t &hc,
                                         uint32_t &hg, uint32_t &f, uint32_t &key,
                                         uint32_t tw, uint32_t tl, uint32_t th, uint32_t end1,
                                         uint32_t begw, uint32_t oe2, uint32_t ed2,
                                         const PkRow &r)
{
    constexpr uint32_t J0 = 4 * G;
    constexpr uint32_t P0 = J0 * 0x10001u, P1 = (J0 + 1) * 0x10001u, P2 = (J0 + 2) * 0x10001u,
                       P3 = (J0 + 3) * 0x10001u, PM = (J0 - 1) * 0x10001u;   // (j, j) packed
    uint32_t m0, m1, m2, m3, t0, t1, t2, t3, x0, x1, x2, x3, ha, ka, mo, mg, ml;
    uint32_t sj, st;
#define PK_P1(K, QP, DUP)                                                                    \
    "v_perm_b32 %[m" #K "], %[" QP "], %[" QP "], %[" DUP "]\n\t"                              \
    PK_ACCR("%[x" #K "]", "%[e" #K "]")                                                       \
    "v_xor_b32 %[m" #K "], %[m" #K "], %[tw]\n\t"                                               \
    "v_perm_b32 %[m" #K "], %[th], %[tl], %[m" #K "]\n\t"                                       \
    "v_pk_min_i16 %[m" #K "], %[m" #K "], %[h" #K "]\n\t"                                       \
    "v_pk_add_u16 %[m" #K "], %[m" #K "], %[h" #K "]\n\t"                                       \
    "v_pk_sub_i16 %[t" #K "], %[m" #K "], %[oe2]\n\t"                                           \
    "v_pk_max_i16 %[t" #K "], %[t" #K "], 0\n\t"                                                \
    "v_pk_max_i16 %[m" #K "], %[m" #K "], %[x" #K "]\n\t"                                       \
    "v_pk_sub_i16 %[x" #K "], %[x" #K "], %[ed2]\n\t"
#define PK_FAST(K, HOUT, PJ)                                                             \
    "v_pk_max_i16 %[x" #K "], %[x" #K "], %[t" #K "]\n\t"                                       \
    PK_ACCW("%[e" #K "]", "%[x" #K "]")                                                       \
    "v_pk_max_i16 " HOUT ", %[m" #K "], %[f]\n\t"                                               \
    "v_pk_sub_i16 %[f], %[f], %[ed2]\n\t"                                                       \
    "v_pk_max_i16 %[f], %[f], %[t" #K "]\n\t"                                                   \
    "v_pk_lshlrev_b16 %[ka], 8, " HOUT " op_sel_hi:[0,1]\n\t"                                  \
    "v_or_b32 %[ka], %[" PJ "], %[ka]\n\t"                                                      \
    "v_pk_max_u16 %[key], %[key], %[ka]\n\t"
    // masked cell: GTR holds GT (= OUT of the previous column), OUTR receives OUT of this one
#define PK_MASK(K, HOUT, HOLD, PJ, GTR, OUTR)                                            \
    "s_mov_b32 %[sj], %[" PJ "]\n\t"                                                            \
    "v_pk_sub_i16 %[" OUTR "], %[end1], %[sj]\n\t"                                              \
    "v_pk_ashrrev_i16 %[" OUTR "], 15, %[" OUTR "] op_sel_hi:[0,1]\n\t"                        \
    "v_pk_sub_i16 %[ml], %[sj], %[begw]\n\t"                                                    \
    "v_pk_ashrrev_i16 %[ml], 15, %[ml] op_sel_hi:[0,1]\n\t"                                    \
    "v_pk_max_i16 %[x" #K "], %[x" #K "], %[t" #K "]\n\t"                                       \
    "v_bfi_b32 %[x" #K "], %[" OUTR "], 0, %[x" #K "]\n\t"                                      \
    PK_ACCR("%[ha]", "%[e" #K "]")                                                            \
    "v_bfi_b32 %[x" #K "], %[" GTR "], %[ha], %[x" #K "]\n\t"                                  \
    PK_ACCW("%[e" #K "]", "%[x" #K "]")                                                       \
    "v_pk_max_i16 %[ha], %[m" #K "], %[f]\n\t"                                                  \
    "v_bfi_b32 " HOUT ", %[" OUTR "], " HOLD ", %[ha]\n\t"                                     \
    "v_pk_sub_i16 %[f], %[f], %[ed2]\n\t"                                                       \
    "v_pk_max_i16 %[f], %[f], %[t" #K "]\n\t"                                                   \
    "v_bfi_b32 %[f], %[ml], 0, %[f]\n\t"                                                        \
    "v_or_b32 %[ml], %[ml], %[" OUTR "]\n\t"                                                    \
    "v_bfi_b32 %[hg], %[ml], %[hg], %[ha]\n\t"                                                 \
    "v_pk_lshlrev_b16 %[ka], 8, %[ha] op_sel_hi:[0,1]\n\t"                                     \
    "v_or_b32 %[ka], %[" PJ "], %[ka]\n\t"                                                      \
    "v_bfi_b32 %[ka], %[ml], 0, %[ka]\n\t"                                                      \
    "v_pk_max_u16 %[key], %[key], %[ka]\n\t"
    asm volatile(
        PK_TESTS("s_sub_u32 %[st], %[g], %[glo]\n\t"
        "s_cmp_le_u32 %[st], %[gsp]\n\t", "s_cbranch_scc0 3f\n\t")
        PK_ACCR("%[mo]", "%[qa]") PK_ACCR("%[mg]", "%[qb]")
        PK_P1(0, "mo", "d0") PK_P1(1, "mo", "d1") PK_P1(2, "mg", "d0") PK_P1(3, "mg", "d1")
        "v_mov_b32 %[h0], %[hc]\n\t"
        PK_TESTS("s_sub_u32 %[st], %[g], %[gfa]\n\t"
        "s_cmp_lt_u32 %[st], %[gfn]\n\t", "s_cbranch_scc0 2f\n\t")
        PK_FAST(0, "%[h1]", "p0") PK_FAST(1, "%[h2]", "p1")
        PK_FAST(2, "%[h3]", "p2") PK_FAST(3, "%[hc]", "p3")
        "v_mov_b32 %[hg], %[hc]\n\t"
        PK_TESTS("", "s_branch 3f\n")
        PK_SLOW(
        "2:\n\t"
        "s_mov_b32 %[sj], %[pm]\n\t"
        "v_pk_sub_i16 %[mg], %[end1], %[sj]\n\t"
        "v_pk_ashrrev_i16 %[mg], 15, %[mg] op_sel_hi:[0,1]\n\t"
        PK_MASK(0, "%[h1]", "%[h1]", "p0", "mg", "mo")
        PK_MASK(1, "%[h2]", "%[h2]", "p1", "mo", "mg")
        PK_MASK(2, "%[h3]", "%[h3]", "p2", "mg", "mo")
        PK_MASK(3, "%[hc]", "%[hn]", "p3", "mo", "mg"))
        "3:\n\t"
        : [h0] "+v"(h0), [h1] "+v"(h1), [h2] "+v"(h2), [h3] "+v"(h3), [e0] PK_ECON(e0), [e1] PK_ECON(e1),
          [e2] PK_ECON(e2), [e3] PK_ECON(e3), [hc] "+v"(hc), [hg] "+v"(hg), [f] "+v"(f), [key] "+v"(key),
          [m0] "=&v"(m0), [m1] "=&v"(m1), [m2] "=&v"(m2), [m3] "=&v"(m3),
          [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [x0] "=&v"(x0),
          [x1] "=&v"(x1), [x2] "=&v"(x2), [x3] "=&v"(x3), [ha] "=&v"(ha), [ka] "=&v"(ka),
          [mo] "=&v"(mo), [mg] "=&v"(mg), [ml] "=&v"(ml), [sj] "=&s"(sj),
          [st] "=&s"(st)
        : [hn] "v"(hn), [qa] PK_QCON(qa), [qb] PK_QCON(qb), [tw] "v"(tw), [tl] "v"(tl), [th] "v"(th),
          [end1] "v"(end1), [begw] "v"(begw), [oe2] "s"(oe2), [ed2] "s"(ed2),
          [d0] "s"(0x01010000u), [d1] "s"(0x03030202u), [g] "i"(G), [glo] "s"(r.glo),
          [gsp] "s"(r.gsp), [gfa] "s"(r.gfa), [gfn] "s"(r.gfn), [p0] "i"(P0), [p1] "i"(P1),
          [p2] "i"(P2), [p3] "i"(P3), [pm] "i"(PM)
        : "scc");
#undef PK_P1
#undef PK_FAST
#undef PK_MASK
}

template <int QMAX, int... G>
__device__ __forceinline__ void pk_row(std::integer_sequence<int, G...>, uint32_t (&hh)[QMAX + 1],
                                       uint32_t (&ee)[QMAX], const uint32_t (&qp)[QMAX / 2],
                                       uint32_t &hc, uint32_t &hg, uint32_t &f, uint32_t &key,
                                       uint32_t tw, uint32_t tl, uint32_t th,
                                       uint32_t end1, uint32_t begw, uint32_t oe2, uint32_t ed2,
                                       const PkRow &r)
{
    (pk_group<G>(hh[4 * G], hh[4 * G + 1], hh[4 * G + 2], hh[4 * G + 3], ee[4 * G], ee[4 * G + 1],
                 ee[4 * G + 2], ee[4 * G + 3], hh[4 * G + 4], qp[2 * G], qp[2 * G + 1], hc, hg, f,
                 key, tw, tl, th, end1, begw, oe2, ed2, r),
     ...);
}

// Row-end bookkeeping of one pair (A.4 tail): gscore at j == qlen, m == 0 termination, new
// best, z-drop, next end = min(last positive + 3, qlen).
__device__ __forceinline__ void pk_row_end(PkHalf &s, int i, int end, uint32_t key16,
                                           uint32_t hg16, const KParams &kp)
{
    const int m = (int)(key16 >> 8), mj = (int)(key16 & 0xffu);
    const int h1 = (int)hg16;
    if (end == s.qlen) {
        if (!(s.gsc > h1)) s.max_ie = i;
        s.gsc = max(s.gsc, h1);
    }
    if (m <= 0) {
        s.alive = false;
    } else if (m > s.best) {
        s.best = m; s.best_i = i; s.best_j = mj;
        s.moff = max(s.moff, abs(mj - i));
    } else if (kp.zdrop > 0) {
        const int di = i - s.best_i, dj = mj - s.best_j;
        const int dz = (di > dj) ? s.best - m - (di - dj) * kp.e_del : s.best - m - (dj - di) * kp.e_ins;
        if (dz > kp.zdrop) s.alive = false;
    }
}

// Lazy last positive column (as the lane kernel's lane_lastpos): for the pairs whose
// H(i, end-1) is 0, scan HH[j+1] = H(i, j) right to left from end - 1 (per half).
template <int QMAX, int GG>
__device__ __forceinline__ void pk_lastpos_group(const uint32_t (&hh)[QMAX + 1], const int (&end)[2],
                                                 bool (&pend)[2], int (&lp1)[2], int gstart)
{
    if (GG > gstart) return;                                           // uniform
    if (__ballot(pend[0] || pend[1]) == 0) return;                     // uniform
#pragma unroll
    for (int k = 3; k >= 0; --k) {
        const int j = 4 * GG + k;
        if (j < QMAX) {
            const uint32_t v = hh[j + 1];          // branch-free selects (no EXEC splits)
            const bool a = pend[0] & (j < end[0]) & ((v & 0xffffu) != 0u);
            const bool b = pend[1] & (j < end[1]) & ((v >> 16) != 0u);
            lp1[0] = a ? j + 1 : lp1[0];
            lp1[1] = b ? j + 1 : lp1[1];
            pend[0] = pend[0] & !a;
            pend[1] = pend[1] & !b;
        }
    }
}

template <int QMAX, int... G>
__device__ __forceinline__ void pk_lastpos(std::integer_sequence<int, G...>, const uint32_t (&hh)[QMAX + 1],
                                           const int (&end)[2], bool (&pend)[2], int (&lp1)[2], int gstart)
{
    (pk_lastpos_group<QMAX, QMAX / 4 - 1 - G>(hh, end, pend, lp1, gstart), ...);
}

// Row-target encoding for the score XOR: lo selector t (N: 8), hi selector t ^ 12 (N: 5 ^ 12).
__device__ __forceinline__ uint32_t pk_tenc(uint32_t t)
{
    return t < 4u ? (t | ((t ^ 12u) << 8)) : (8u | (9u << 8));
}

// QMAX <= 64 fits two waves per SIMD (<= 256 VGPR + AGPR); larger buckets run one.
template <int QMAX>
__global__ __launch_bounds__(256, QMAX <= 64 ? 2 : 1) void pk_kernel(const KParams kp, const int32_t w,
                                                    SeqPair *__restrict__ pairs,
                                                    const int32_t *__restrict__ order,
                                                    const int32_t n,
                                                    const uint8_t *__restrict__ ref,
                                                    const uint8_t *__restrict__ qer,
                                                    int32_t *__restrict__ err)
{
    static_assert(QMAX % 4 == 0 && QMAX <= 252, "QMAX");
    constexpr int NG = QMAX / 4;
    __shared__ uint32_t s_tgt[4][2][2][kPkChunkDw][64];   // [wave][pair][buffer][dword][lane]
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int base = (blockIdx.x * 4 + wv) * 128;
    PkHalf hs[2];
    const uint8_t *tpp[2];
    int tsh[2], tlast[2];
    const uint32_t *twp[2];
    uint32_t qw[2][NG];
    SeqPair *sp[2];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        PkHalf &s = hs[hf];
        const int gid = base + hf * 64 + ln;
        s.valid = gid < n;
        const int idx = s.valid ? order[gid] : 0;
        sp[hf] = pairs + idx;
        int idr = 0, idq = 0;
        s.tlen = s.qlen = s.h0 = 0;
        if (s.valid) {
            const SeqPair &p = *sp[hf];
            idr = p.idr; idq = p.idq; s.tlen = p.len1; s.qlen = p.len2; s.h0 = p.h0;
            if (s.qlen > QMAX || s.qlen < 0 || s.tlen < 0 || s.h0 < 0 || s.h0 + min(s.qlen, s.tlen) > 255) {
                atomicOr(err, 2);
                s.valid = false;
                s.tlen = s.qlen = s.h0 = 0;
            }
        }
        // query codes: aligned dword loads (page-safe), realigned with v_alignbyte
        {
            uint32_t wd[NG + 1];
            const uintptr_t qa = (uintptr_t)(qer + idq);
            const uint32_t *wp = (const uint32_t *)(qa & ~(uintptr_t)3);
            const int sh = (int)(qa & 3);
            const int nw = (s.valid && s.qlen > 0) ? (sh + s.qlen + 3) >> 2 : 0;
            if (nw > 0) {
#pragma unroll
                for (int g = 0; g <= NG; ++g) wd[g] = wp[min(g, nw - 1)];
            } else {
#pragma unroll
                for (int g = 0; g <= NG; ++g) wd[g] = 0;
            }
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                uint32_t c = __builtin_amdgcn_alignbyte(wd[g + 1], wd[g], sh);
                c = c + ((c & 0x04040404u) >> 1);          // code N (4) -> 6, ACGT unchanged
                qw[hf][g] = c;
            }
        }
        // band cap (A.2), integer form
        int wl = w;
        {
            const int ni = s.qlen * kp.maxsc + kp.end_bonus - kp.o_ins;
            const int nd = s.qlen * kp.maxsc + kp.end_bonus - kp.o_del;
            wl = min(wl, max((ni + kp.e_ins) / kp.e_ins, 1));
            wl = min(wl, max((nd + kp.e_del) / kp.e_del, 1));
        }
        s.wl = wl;
        s.best = s.h0; s.best_i = -1; s.best_j = -1; s.max_ie = -1; s.gsc = -1; s.moff = 0;
        s.endc = s.qlen;
        s.alive = s.valid && s.tlen > 0;
        tpp[hf] = ref + idr;
        tsh[hf] = (int)((uintptr_t)tpp[hf] & 3);
        twp[hf] = (const uint32_t *)(tpp[hf] - tsh[hf]);
        tlast[hf] = max((tsh[hf] + s.tlen - 1) >> 2, 0);
    }
    // query words of the two pairs interleaved: qp[2g] = {A_4g, B_4g, A_4g+1, B_4g+1}
    uint32_t qp[QMAX / 2];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        qp[2 * g] = __builtin_amdgcn_perm(qw[1][g], qw[0][g], 0x05010400u);
        qp[2 * g + 1] = __builtin_amdgcn_perm(qw[1][g], qw[0][g], 0x07030602u);
    }
    __builtin_amdgcn_sched_barrier(0);
    // A.1 first row, both pairs: H(-1, j-1) = max(h0 - oe_ins - (j-1) e_ins, 0), E = 0
    uint32_t hh[QMAX + 1], ee[QMAX];
    {
        const int oe_ins = kp.o_ins + kp.e_ins;
        hh[0] = (uint32_t)hs[0].h0 | ((uint32_t)hs[1].h0 << 16);
#pragma unroll
        for (int j = 1; j <= QMAX; ++j) {
            const uint32_t a = (j <= hs[0].qlen) ? (uint32_t)max(hs[0].h0 - oe_ins - (j - 1) * kp.e_ins, 0) : 0u;
            const uint32_t b = (j <= hs[1].qlen) ? (uint32_t)max(hs[1].h0 - oe_ins - (j - 1) * kp.e_ins, 0) : 0u;
            hh[j] = a | (b << 16);
        }
#pragma unroll
        for (int j = 0; j < QMAX; ++j) ee[j] = 0;
    }
    // target streams: both pairs' bases HBM -> LDS by LDS-DMA, 64-row chunks double-buffered
    auto issue_chunk = [&](int hf, int ch) {
        uint32_t *dst = &s_tgt[wv][hf][ch & 1][0][0];
#pragma unroll
        for (int k = 0; k < kPkChunkDw; ++k)
            __builtin_amdgcn_global_load_lds((gptr_t)(twp[hf] + min(16 * ch + k, tlast[hf])),
                                             (lptr_t)(dst + 64 * k), 4, 0, 0);
    };
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
        if (hs[hf].alive) { issue_chunk(hf, 0); issue_chunk(hf, 1); }
    const int wl_max = wave_max(max(hs[0].alive ? hs[0].wl : -1, hs[1].alive ? hs[1].wl : -1));
    const int wl_min = wave_min(min(hs[0].alive ? hs[0].wl : INT_MAX, hs[1].alive ? hs[1].wl : INT_MAX));
    const uint32_t oe2 = (uint32_t)(kp.o_del + kp.e_del) * 0x10001u;
    const uint32_t ed2 = (uint32_t)kp.e_del * 0x10001u;
    const uint32_t tl = 1u | ((uint32_t)(uint8_t)kp.mat[1] * 0x01010100u);   // {a, -b, -b, -b}
    const uint32_t th = 0xffffffffu;                                          // N: -1
    uint32_t tcur[2] = {0u, 0u};
#ifdef BSW_PK_STAMPS   // diagnostic builds only: per-phase cycle totals (tools/pk_stamps.py)
    uint32_t acc[5] = {0u, 0u, 0u, 0u, 0u};
    uint64_t ts0, ts1;
#define PK_STAMP(k) do { ts1 = __builtin_amdgcn_s_memtime(); acc[k] += (uint32_t)(ts1 - ts0); ts0 = ts1; } while (0)
    ts0 = __builtin_amdgcn_s_memtime();
#else
#define PK_STAMP(k) do { } while (0)
#endif

    for (int i = 0;; ++i) {
        bool act2[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            act2[hf] = hs[hf].alive && i < hs[hf].tlen;
            hs[hf].alive = act2[hf];
        }
        const bool act = act2[0] || act2[1];
        if (__ballot(act) == 0) break;
        int beg[2], end[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            beg[hf] = max(0, i - hs[hf].wl);
            end[hf] = min(min(hs[hf].endc, i + hs[hf].wl + 1), hs[hf].qlen);
            hs[hf].endc = end[hf];
        }
        PK_STAMP(0);
        const int emax = wave_max(max(act2[0] ? end[0] : -1, act2[1] ? end[1] : -1));
        const int emin = wave_min(min(act2[0] ? end[0] : INT_MAX, act2[1] ? end[1] : INT_MAX));
        PkRow r;
        {
            const int ulo = __builtin_amdgcn_readfirstlane(max(0, i - wl_max));
            const int uhi = __builtin_amdgcn_readfirstlane(emax);
            const int flo = __builtin_amdgcn_readfirstlane(max(0, i - wl_min));
            const int fhi = __builtin_amdgcn_readfirstlane(emin);
            r.glo = ulo >> 2;
            r.gsp = max(min(uhi, QMAX - 1) / 4 - r.glo, -1);
            r.gfa = (flo + 3) >> 2;
            r.gfn = max((fhi >> 2) - r.gfa, 0);
        }
        PK_STAMP(1);
        if (act) {
            if ((i & 3) == 0) {               // 4 target bases per pair from LDS
                if ((i & 63) == 0) {
                    __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0)
                    __builtin_amdgcn_sched_barrier(0);
                }
                const int k = (i >> 2) & 15;
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    const uint32_t *src = &s_tgt[wv][hf][(i >> 6) & 1][k][ln];
                    tcur[hf] = __builtin_amdgcn_alignbyte(src[64], src[0], tsh[hf]);
                }
                if ((i & 63) == 0) {
                    __builtin_amdgcn_sched_barrier(0);
                    if (i > 0) {
#pragma unroll
                        for (int hf = 0; hf < 2; ++hf)
                            if (hs[hf].alive) issue_chunk(hf, (i >> 6) + 1);
                    }
                }
            }
            const uint32_t ta = min((tcur[0] >> (8 * (i & 3))) & 0xffu, 4u);
            const uint32_t tb = min((tcur[1] >> (8 * (i & 3))) & 0xffu, 4u);
            const uint32_t tw = pk_tenc(ta) | (pk_tenc(tb) << 16);
            uint32_t hc;
            {
                const int bA = (beg[0] == 0) ? max(hs[0].h0 - (kp.o_del + kp.e_del * (i + 1)), 0) : 0;
                const int bB = (beg[1] == 0) ? max(hs[1].h0 - (kp.o_del + kp.e_del * (i + 1)), 0) : 0;
                hc = (uint32_t)bA | ((uint32_t)bB << 16);
            }
            uint32_t hg = hc, f = 0, key = 0;
            const uint32_t end1 = ((uint32_t)(end[0] - 1) & 0xffffu) | ((uint32_t)(end[1] - 1) << 16);
            const uint32_t begw = (uint32_t)beg[0] | ((uint32_t)beg[1] << 16);
            PK_STAMP(2);
            pk_row<QMAX>(std::make_integer_sequence<int, NG>{}, hh, ee, qp, hc, hg, f, key, tw, tl,
                         th, end1, begw, oe2, ed2, r);
            PK_STAMP(3);
            if (act2[0]) pk_row_end(hs[0], i, end[0], key & 0xffffu, hg & 0xffffu, kp);
            if (act2[1]) pk_row_end(hs[1], i, end[1], key >> 16, hg >> 16, kp);
            // next band end: lastH = end - 1 when H(i, end-1) > 0, else recovered
            bool pend[2] = {act2[0] && hs[0].alive && (hg & 0xffffu) == 0u,
                            act2[1] && hs[1].alive && (hg >> 16) == 0u};
            int lp1[2] = {end[0], end[1]};
            if (__ballot(pend[0] || pend[1])) {
                if (pend[0]) lp1[0] = 0;
                if (pend[1]) lp1[1] = 0;
                pk_lastpos<QMAX>(std::make_integer_sequence<int, NG>{}, hh, end, pend, lp1, (emax - 1) >> 2);
            }
#pragma unroll
            for (int hf = 0; hf < 2; ++hf)
                if (act2[hf] && hs[hf].alive) hs[hf].endc = min(lp1[hf] + 2, hs[hf].qlen);
        }
        PK_STAMP(4);
    }
#ifdef BSW_PK_STAMPS
    if (hs[0].valid) { sp[0]->seqid = (int32_t)acc[0]; sp[0]->regid = (int32_t)acc[1]; sp[0]->id = (int32_t)acc[4]; }
    if (hs[1].valid) { sp[1]->seqid = (int32_t)acc[2]; sp[1]->regid = (int32_t)acc[3]; }
#endif
#undef PK_STAMP
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        const PkHalf &s = hs[hf];
        if (s.valid) {
            SeqPair *p = sp[hf];
            p->score = s.best;
            p->tle = s.best_i + 1;
            p->gtle = s.max_ie + 1;
            p->qle = s.best_j + 1;
            p->gscore = s.gsc;
            p->max_off = s.moff;
        }
    }
}

hipError_t launch_pk_kernel(int qmax, const KParams &kp, int32_t w, SeqPair *pairs,
                            const int32_t *order, int32_t n, const uint8_t *ref,
                            const uint8_t *qer, int32_t *err, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    const dim3 block(256), grid((unsigned)((n + 511) / 512));
    switch (qmax) {
    case 32: hipLaunchKernelGGL(pk_kernel<32>, grid, block, 0, s, kp, w, pairs, order, n, ref, qer, err); break;
    case 64: hipLaunchKernelGGL(pk_kernel<64>, grid, block, 0, s, kp, w, pairs, order, n, ref, qer, err); break;
    case 96: hipLaunchKernelGGL(pk_kernel<96>, grid, block, 0, s, kp, w, pairs, order, n, ref, qer, err); break;
    case 128: hipLaunchKernelGGL(pk_kernel<128>, grid, block, 0, s, kp, w, pairs, order, n, ref, qer, err); break;
    case 160: hipLaunchKernelGGL(pk_kernel<160>, grid, block, 0, s, kp, w, pairs, order, n, ref, qer, err); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace bsw
