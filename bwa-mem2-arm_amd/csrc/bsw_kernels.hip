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

#ifndef BSW_CELL_FENCE
#define BSW_CELL_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif

namespace bsw {

// ------------------------------------------------------------------ wave-level helpers
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
__device__ __forceinline__ int wave_min(int x) { return -wave_max(-x); }

__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

// ------------------------------------------------------------------ lane kernel
struct LaneRow {          // per-row uniform (SGPR) bounds
    int ulo, uhi;         // min beg / max end over live lanes (columns outside: skipped)
    int fast_lo, fast_hi; // max beg / min end over live lanes (columns inside: unmasked)
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

// Row pass structure.  Per row the wave knows, over its live lanes,
//   [flo, fhi)  : columns where EVERY live lane is in band  -> fast pass, no lane masks
//   [elo, ehi]  : remaining columns up to the largest end   -> edge pass, per-lane masks
// Both passes are straight-line unrolled sequences whose columns are guarded only by
// uniform (SGPR) range tests -- no if/else pair ever writes the same eh[] register, so the
// row stays in place in its VGPRs (no merge copies).

// Fast-pass column J.
template <int J, int QMAX, int SM, bool SYM>
__device__ __forceinline__ void lane_col_fast(uint32_t (&eh)[QMAX + 1], uint32_t pw, int &f, int &h1,
                                              int &key, int &lp1, const LaneRow &r, const LaneCx &c)
{
    if constexpr (J < QMAX) {
        if (J >= r.fast_lo && J < r.fast_hi)
            lane_cell<J, SM, SYM, QMAX + 1>(eh, (int)(int8_t)(pw >> (8 * (J & 3))), f, h1, key, lp1, c);
    }
}

// Edge-pass column J: per-lane band membership under EXEC; at j == end write
// { H(i,end-1), 0 } (A.4 end of row); beyond end leave eh untouched (A.7 stale columns).
template <int J, int QMAX, int SM, bool SYM>
__device__ __forceinline__ void lane_col_edge(uint32_t (&eh)[QMAX + 1], const uint32_t (&q4)[QMAX / 4],
                                              uint2 pr, int beg, int end, int &f, int &h1, int &key,
                                              int &lp1, const LaneRow &r, const LaneCx &c)
{
    if (J < r.ulo || J > r.uhi) return;                   // uniform
    if constexpr (J < QMAX) {
        if (J >= beg && J < end) {
            const uint32_t pw = __builtin_amdgcn_perm(pr.y, pr.x, q4[J / 4]);
            lane_cell<J, SM, SYM, QMAX + 1>(eh, (int)(int8_t)(pw >> (8 * (J & 3))), f, h1, key,
                                            lp1, c);
            return;
        }
    }
    if (J == end) eh[J] = (uint32_t)h1;
}

template <int G, int QMAX, int SM, bool SYM>
__device__ __forceinline__ void lane_group_fast(uint32_t (&eh)[QMAX + 1], const uint32_t (&q4)[QMAX / 4],
                                                uint2 pr, int &f, int &h1, int &key, int &lp1,
                                                const LaneRow &r, const LaneCx &c)
{
    constexpr int J0 = 4 * G;
    if constexpr (J0 >= QMAX) return;
    if (J0 + 3 < r.fast_lo || J0 >= r.fast_hi) return;   // uniform skip
    const uint32_t pw = __builtin_amdgcn_perm(pr.y, pr.x, q4[G]);
    lane_col_fast<J0 + 0, QMAX, SM, SYM>(eh, pw, f, h1, key, lp1, r, c);
    lane_col_fast<J0 + 1, QMAX, SM, SYM>(eh, pw, f, h1, key, lp1, r, c);
    lane_col_fast<J0 + 2, QMAX, SM, SYM>(eh, pw, f, h1, key, lp1, r, c);
    lane_col_fast<J0 + 3, QMAX, SM, SYM>(eh, pw, f, h1, key, lp1, r, c);
}

template <int G, int QMAX, int SM, bool SYM>
__device__ __forceinline__ void lane_group_edge(uint32_t (&eh)[QMAX + 1], const uint32_t (&q4)[QMAX / 4],
                                                uint2 pr, int beg, int end, int &f, int &h1,
                                                int &key, int &lp1, const LaneRow &r, const LaneCx &c)
{
    constexpr int J0 = 4 * G;
    if (J0 + 3 < r.ulo || J0 > r.uhi) return;            // uniform skip
    lane_col_edge<J0 + 0, QMAX, SM, SYM>(eh, q4, pr, beg, end, f, h1, key, lp1, r, c);
    if constexpr (J0 + 1 <= QMAX) lane_col_edge<J0 + 1, QMAX, SM, SYM>(eh, q4, pr, beg, end, f, h1, key, lp1, r, c);
    if constexpr (J0 + 2 <= QMAX) lane_col_edge<J0 + 2, QMAX, SM, SYM>(eh, q4, pr, beg, end, f, h1, key, lp1, r, c);
    if constexpr (J0 + 3 <= QMAX) lane_col_edge<J0 + 3, QMAX, SM, SYM>(eh, q4, pr, beg, end, f, h1, key, lp1, r, c);
}

template <int QMAX, int SM, bool SYM, int... G>
__device__ __forceinline__ void lane_row(std::integer_sequence<int, G...>, uint32_t (&eh)[QMAX + 1],
                                         const uint32_t (&q4)[QMAX / 4], uint2 pr, int beg, int end,
                                         int &f, int &h1, int &key, int &lp1, const LaneRow &fast,
                                         const LaneRow &edge, const LaneCx &c)
{
    (lane_group_fast<G, QMAX, SM, SYM>(eh, q4, pr, f, h1, key, lp1, fast, c), ...);
    (lane_group_edge<G, QMAX, SM, SYM>(eh, q4, pr, beg, end, f, h1, key, lp1, edge, c), ...);
}

__device__ __forceinline__ uint32_t load4(const uint8_t *p, int base, int len)
{
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + k < len) w |= (uint32_t)p[base + k] << (8 * k);
    return w;
}

template <int QMAX, int SM, bool SYM>
__global__ __launch_bounds__(256, 2) void lane_kernel(const KParams kp, const int32_t w,
                                                      SeqPair *__restrict__ pairs,
                                                      const int32_t *__restrict__ order,
                                                      const int32_t n,
                                                      const uint8_t *__restrict__ ref,
                                                      const uint8_t *__restrict__ qer,
                                                      int32_t *__restrict__ err)
{
    constexpr int NG = QMAX / 4;        // query words (4 codes each)
    __shared__ uint2 tab[8];
    if (threadIdx.x < 8) tab[threadIdx.x] = make_uint2(kp.prof[threadIdx.x][0], kp.prof[threadIdx.x][1]);
    __syncthreads();

    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = gid < n;
    const int idx = valid ? (order ? order[gid] : gid) : 0;
    SeqPair *sp = pairs + idx;
    int idr = 0, idq = 0, tlen = 0, qlen = 0, h0 = 0;
    if (valid) {
        idr = sp->idr; idq = sp->idq; tlen = sp->len1; qlen = sp->len2; h0 = sp->h0;
        if (qlen > QMAX || qlen < 0 || tlen < 0) { atomicOr(err, 1); valid = false; }
    }
    // query codes -> perm selectors (codes > 7 clamp to 7 = ambig slot)
    uint32_t q4[NG];
    const uint8_t *qp = qer + idq;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        uint32_t word = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = 4 * g + k;
            if (valid && j < qlen) word |= (uint32_t)min((uint32_t)qp[j], 7u) << (8 * k);
        }
        q4[g] = word;
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
    const uint8_t *tp = ref + idr;
    uint32_t tcur = 0, tnxt = 0;
    if (alive) { tcur = load4(tp, 0, tlen); tnxt = load4(tp, 4, tlen); }
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
        LaneRow fast, edge;
        if (wl_min == wl_max) {
            fast.fast_lo = max(0, i - wl_min);
            fast.fast_hi = emin;
            edge.ulo = max(fast.fast_lo, emin);
        } else {
            fast.fast_lo = fast.fast_hi = 0;
            edge.ulo = max(0, i - wl_max);
        }
        edge.uhi = emax;
        if (act) {
            if ((i & 3) == 0 && i > 0) { tcur = tnxt; tnxt = load4(tp, i + 4, tlen); }
            const uint32_t t = min((tcur >> (8 * (i & 3))) & 0xffu, 7u);
            const uint2 pr = tab[t];
            int h1 = (beg == 0) ? max(h0 - (kp.o_del + kp.e_del * (i + 1)), 0) : 0;
            int f = 0, key = -1, lp1 = 0;
            lane_row<QMAX, SM, SYM>(std::make_integer_sequence<int, QMAX / 4 + 1>{}, eh, q4, pr,
                                    beg, end, f, h1, key, lp1, fast, edge, cx);
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
            if (alive) endc = min(lp1 + 2, qlen);   // = min(last nonzero eh + 2, qlen), DESIGN.md §3
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
    const dim3 block(256), grid((unsigned)((n + 255) / 256));
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
