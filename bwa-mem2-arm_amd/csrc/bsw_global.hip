// bsw_global.hip -- CDNA4 (gfx950) batch kernels for banded GLOBAL alignment with traceback:
// upstream ksw_global2 semantics (include/bsw_global.h).
//
// Register kernel (glob_lane_kernel<QMAX>): one LANE per job, as the extension lane kernel
// (bsw_kernels.hip).  The job's DP row eh[0..qlen) lives in VGPRs as packed {h:16, e:16} per
// query column -- eh[j] = {H(i-1, j-1), E(i, j)} at the start of row i -- query codes 4 per
// VGPR, per-row scores by v_perm from the 8-byte profile of the row's target base.  A
// wavefront advances 64 jobs through their target rows in lock-step.  Columns are handled in
// groups of 8: groups outside every lane's band [max(i - w, 0), min(i + w + 1, qlen)] (+ the
// column `end` that receives eh[end] = {h1, -inf}) are skipped by scalar tests, groups inside
// every band run unmasked, the rest with per-lane selects.  -inf is -16384 in the int16 row
// (the planner sends jobs whose scores could leave +-15000 to the wide kernel), so every
// comparison between a -inf-derived and a finite value has the same outcome as upstream's
// int32 MINUS_INF = -0x40000000; the returned score keeps upstream's value.
//
// Traceback matrix: ksw_global2 keeps a byte per band cell (h direction | E bit << 2 | F bit
// << 4); here a nibble (h direction 0..2 | E bit << 2 | F bit << 3), 8 columns per dword, in
// HBM per wavefront as [row][dword window][lane], so each row's store of one dword is one
// coalesced 256-byte line.  The window of row i starts at dword max(i - wmax, 0) >> 3 (wmax =
// the wave's widest band) and holds cap_dw dwords (glob_cap_dw), enough for every lane's band.
// After the last row each lane walks its own path back through its nibbles (upstream's
// `which` state machine) and writes the run-length CIGAR, reversed in place at the end.
//
// Wide kernel (glob_wide_kernel): the literal int32 row code per lane with eh[] in HBM scratch
// laid out [column][slot] (coalesced across the wave), the same traceback matrix layout and the
// same traceback -- qlen > 160 or scores that do not fit the int16 row.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include <utility>
#include "bsw_global_k.h"
#include "bsw_wave.h"

namespace bsw {

constexpr int kGNeg = -16384;                 // -inf of the int16 register rows
constexpr int32_t kGMinusInf = -0x40000000;   // upstream MINUS_INF

// Routing: the column kernel when the job fits it (measured faster on bwa-shaped jobs: 9.55 vs
// 9.76 ms per 1M 150-bp jobs), else the band kernel when 2w + 2 <= 96, else the wide kernel;
// gp.prefer_band (BSW_OPT_GLOB_BAND) puts every band-eligible job on the band kernel.
__device__ __forceinline__ int glob_class(const SeqPair &p, const GlobParams &gp)
{
    const int q = p.len2, t = p.len1, w = p.h0;
    if (q < 0 || t < 0 || w < 0 || q > BSW_MAX_LEN || t > BSW_MAX_LEN) return -1;
    // every finite cell value lies within +-bound (diagonal run + one gap to any band cell,
    // the row-0 / column-0 boundaries, one more gap open for E' / F')
    const int64_t bound = (int64_t)gp.maxabs * min(q, t) + gp.o_del + (int64_t)gp.e_del * (t + 1) +
                          gp.o_ins + (int64_t)gp.e_ins * (q + 1) + max(gp.oe_del, gp.oe_ins) + 8;
    int col = -1;
    if (bound < 15000) {
        if (q <= 32) col = 0;
        else if (q <= 64) col = 1;
        else if (q <= 96) col = 2;
        else if (q <= 128) col = 3;
        else if (q <= 160) col = 4;
    }
    const int need = 2 * w + 2;                          // band slots incl. the end slot
    int band = -1, bw = 0;
    if (need <= 32) { band = 0; bw = 32; }
    else if (need <= 48) { band = 1; bw = 48; }
    else if (need <= 64) { band = 2; bw = 64; }
    else if (need <= 80) { band = 3; bw = 80; }
    else if (need <= 96) { band = 4; bw = 96; }
    (void)bw;
    if (band >= 0 && (col < 0 || gp.prefer_band)) return band;
    return col >= 0 ? kGlobLane0 + col : kGlobWideClass;
}

__global__ void glob_plan_kernel(const SeqPair *__restrict__ pairs, int32_t n, const GlobParams gp,
                                 uint32_t *__restrict__ keys, int32_t *__restrict__ vals,
                                 int32_t *__restrict__ meta)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int c = -1;
    SeqPair p{};
    if (i < n) {
        p = pairs[i];
        c = glob_class(p, gp);
        if (c < 0) {
            atomicOr(&meta[kGMetaErr], 1);                  // slot 0 (rare)
            c = kGlobWideClass;
        }
        keys[i] = ((uint32_t)c << 28) | ((uint32_t)(1023 - min(max(p.h0, 0), 1023)) << 18) |
                  ((uint32_t)(255 - min(max(p.len2, 0), 255)) << 10) | (uint32_t)(1023 - min(max(p.len1, 0), 1023));
        vals[i] = i;
    }
    // class statistics: per wave (ballot / DPP max) -> per block in LDS -> one global atomic per
    // block, class and statistic into slot blockIdx % kGMetaSpread (slots in separate lines)
    __shared__ int s_st[4][kGlobClasses];
    if (threadIdx.x < 4 * kGlobClasses) (&s_st[0][0])[threadIdx.x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    for (int k = 0; k < kGlobClasses; ++k) {
        const bool mine = c == k;
        const unsigned long long m = __ballot(mine);
        if (!m) continue;                                   // uniform
        const int tm = wave_max(mine ? p.len1 : 0), wm = wave_max(mine ? p.h0 : 0);
        const int qm = wave_max(mine ? p.len2 : 0);
        if (lane == 0) {
            atomicAdd(&s_st[0][k], __popcll(m));
            atomicMax(&s_st[1][k], tm);
            atomicMax(&s_st[2][k], wm);
            atomicMax(&s_st[3][k], qm);
        }
    }
    __syncthreads();
    if (threadIdx.x < kGlobClasses && s_st[0][threadIdx.x]) {
        const int k = threadIdx.x;
        int32_t *slot = meta + (blockIdx.x % kGMetaSpread) * kGMetaWordsPerSlot;
        atomicAdd(&slot[kGMetaCount + k], s_st[0][k]);
        atomicMax(&slot[kGMetaTmax + k], s_st[1][k]);
        atomicMax(&slot[kGMetaWmax + k], s_st[2][k]);
        atomicMax(&slot[kGMetaQmax + k], s_st[3][k]);
    }
}

// ------------------------------------------------------------------ traceback (both kernels)
// zw: this wave's matrix; upstream's loop from (tlen - 1, min(tlen + w, qlen) - 1).
// Narrow window (tb_dw > 0, column kernel): row i holds the tb_dw dwords from column
// max(i + doff, 0) rounded down; a step outside them appends the job to retry (count retry[0]).
__device__ void glob_traceback(const uint32_t *__restrict__ zw, int cap_dw, int wmax, int lane, int qlen,
                               int tlen, int w, uint32_t *__restrict__ out, int stride,
                               int32_t *__restrict__ nout, int tb_dw = 0, int doff = 0,
                               int32_t *__restrict__ retry = nullptr, int idx = 0)
{
    if (qlen >= 1 && tlen >= 1 && qlen < tlen - w) { *nout = -2; return; }
    const int rowdw = tb_dw > 0 ? tb_dw : cap_dw;
    int i = tlen - 1, k = min(i + w + 1, qlen) - 1, which = 0, n = 0;
    uint32_t cur = 0;                                      // last op, not yet stored
    auto push = [&](uint32_t op, uint32_t len) {
        if (n > 0 && (cur & 0xfu) == op) { cur += len << 4; return; }
        if (n > 0 && n - 1 < stride) out[n - 1] = cur;
        cur = len << 4 | op;
        ++n;
    };
    while (i >= 0 && k >= 0) {
        int sl;
        if (tb_dw > 0) {
            sl = (k >> 3) - (max(i + doff, 0) >> 3);
            if ((unsigned)sl >= (unsigned)tb_dw) {           // the path left the corridor
                retry[1 + atomicAdd(retry, 1)] = idx;
                *nout = -3;
                return;
            }
        } else {
            sl = (k >> 3) - (max(i - wmax, 0) >> 3);
        }
        const uint32_t word = zw[((int64_t)i * rowdw + sl) * 64 + lane];
        const uint32_t nib = (word >> ((k & 7) * 4)) & 15u;
        which = which == 0 ? (int)(nib & 3u) : which == 1 ? (int)((nib >> 2) & 1u) : ((nib & 8u) ? 2 : 0);
        if (which == 0) { push(0, 1); --i; --k; }
        else if (which == 1) { push(2, 1); --i; }
        else { push(1, 1); --k; }
    }
    if (i >= 0) push(2, (uint32_t)(i + 1));
    if (k >= 0) push(1, (uint32_t)(k + 1));
    if (n > 0 && n - 1 < stride) out[n - 1] = cur;
    if (n > stride) { *nout = -1; return; }
    for (int a = 0, b = n - 1; a < b; ++a, --b) {
        const uint32_t t = out[a];
        out[a] = out[b];
        out[b] = t;
    }
    *nout = n;
}

// ------------------------------------------------------------------ register kernel
struct GCx {
    int e_del, oe_del, e_ins, oe_ins;
};

// One cell.  R = eh[j] = {H(i-1, j-1), E(i, j)} in, {H(i, j-1), E(i+1, j)} out; h1 = H(i, j-1)
// in, H(i, j) out; f = F(i, j) in, F(i, j+1) out.  Masked: columns outside [beg, end) keep
// everything, column end takes eh[end] = {h1, -inf}.  Returns the direction nibble.
template <bool MASKED>
__device__ __forceinline__ uint32_t glob_cell(uint32_t &R, int s, int &h1, int &f, const GCx &c, bool in,
                                              bool atend)
{
    const int hd = (int)(int16_t)(R & 0xffffu), e = (int)(int16_t)(R >> 16);
    const int m = hd + s;
    int h = max(m, e);
    uint32_t d = m < e ? 1u : 0u;
    d = h < f ? 2u : d;
    h = max(h, f);
    const int t = m - c.oe_del, ee = e - c.e_del;
    const uint32_t eb = ee > t ? 4u : 0u;
    const int e2 = max(ee, t);
    const int t2 = m - c.oe_ins, ff = f - c.e_ins;
    const uint32_t fb = ff > t2 ? 8u : 0u;
    const int f2 = max(ff, t2);
    const uint32_t rn = ((uint32_t)h1 & 0xffffu) | ((uint32_t)e2 << 16);
    if (!MASKED) {
        R = rn; h1 = h; f = f2;
    } else {
        R = in ? rn : (atend ? (((uint32_t)h1 & 0xffffu) | ((uint32_t)kGNeg << 16)) : R);
        h1 = in ? h : h1;
        f = in ? f2 : f;
    }
    return d | eb | fb;
}

template <int G, int QMAX, bool MASKED>
__device__ __forceinline__ uint32_t glob_group(uint32_t (&R)[QMAX], const uint32_t (&q8)[QMAX / 8], uint2 pr,
                                               int &h1, int &f, const GCx &c, int beg, int end)
{
    // q8[G]: codes of columns 8G..8G+7 as nibbles; even columns -> bytes of sel0, odd -> sel1
    const uint32_t sel0 = q8[G] & 0x0f0f0f0fu, sel1 = (q8[G] >> 4) & 0x0f0f0f0fu;
    const uint32_t pw0 = __builtin_amdgcn_perm(pr.y, pr.x, sel0), pw1 = __builtin_amdgcn_perm(pr.y, pr.x, sel1);
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int j = 8 * G + k;
        const int s = (int)(int8_t)(((k & 1) ? pw1 : pw0) >> (8 * (k >> 1)));
        const bool in = MASKED ? (j >= beg && j < end) : true;
        const bool atend = MASKED ? (j == end) : false;
        word |= glob_cell<MASKED>(R[j], s, h1, f, c, in, atend) << (4 * k);
    }
    return word;
}

struct GRow {                       // per-row uniform bounds (SGPRs)
    int lo, hi;                     // columns any lane touches: [min beg, max end + 1)
    int fb, fe;                     // columns every active lane has in band: [max beg, min end)
    int dlo, cap_dw;                // traceback window of this row
    int tb_dw;                      // > 0: narrow per-lane corridor window of tb_dw dwords
};

template <int G, int QMAX>
__device__ __forceinline__ void glob_group_at(uint32_t (&R)[QMAX], const uint32_t (&q8)[QMAX / 8], uint2 pr,
                                              int &h1, int &f, const GCx &c, int beg, int end, const GRow &r,
                                              uint32_t *__restrict__ zrow, int lane, int tlo)
{
    if (8 * G + 8 <= r.lo || 8 * G >= r.hi) return;       // uniform
    uint32_t word;
    if (8 * G >= r.fb && 8 * G + 8 <= r.fe) word = glob_group<G, QMAX, false>(R, q8, pr, h1, f, c, beg, end);
    else word = glob_group<G, QMAX, true>(R, q8, pr, h1, f, c, beg, end);
    if (zrow) {
        if (r.tb_dw > 0) {                                  // narrow: this lane's corridor dwords only
            if ((unsigned)(G - tlo) < (unsigned)r.tb_dw) zrow[(G - tlo) * 64 + lane] = word;
        } else if (G - r.dlo < r.cap_dw) {
            zrow[(G - r.dlo) * 64 + lane] = word;
        }
    }
    // keep the scheduler from interleaving groups: each group's temporaries die here, so the
    // row (QMAX packed {h, e} registers) plus one group's working set fits 2 waves per SIMD
    __builtin_amdgcn_sched_barrier(0);
}

template <int QMAX, int... G>
__device__ __forceinline__ void glob_row(std::integer_sequence<int, G...>, uint32_t (&R)[QMAX],
                                         const uint32_t (&q8)[QMAX / 8], uint2 pr, int &h1, int &f, const GCx &c,
                                         int beg, int end, const GRow &r, uint32_t *__restrict__ zrow, int lane,
                                         int tlo)
{
    (glob_group_at<G, QMAX>(R, q8, pr, h1, f, c, beg, end, r, zrow, lane, tlo), ...);
}

template <int QMAX>
__global__ __launch_bounds__(64, 2) void glob_lane_kernel(
    const GlobParams gp, SeqPair *__restrict__ pairs, const int32_t *__restrict__ order, int32_t n,
    const uint8_t *__restrict__ ref, const uint8_t *__restrict__ qer, uint32_t *__restrict__ z, int64_t zstride,
    int32_t cap_dw, uint32_t *__restrict__ cigar, int32_t stride, int32_t *__restrict__ n_cigar,
    unsigned long long *__restrict__ cells, int32_t tb_dw, int32_t *__restrict__ retry)
{
    constexpr int NG = QMAX / 8;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool live = tid < n;
    const int idx = live ? order[tid] : 0;
    SeqPair p{};
    if (live) p = pairs[idx];
    const int qlen = live ? p.len2 : 0, tlen = live ? p.len1 : 0, w = live ? p.h0 : 0;
    const int wmax = __builtin_amdgcn_readfirstlane(wave_max(live ? w : -1));
    if (wmax < 0) return;                                   // whole wave empty
    const int tmax = __builtin_amdgcn_readfirstlane(wave_max(tlen));
    const int qmw = __builtin_amdgcn_readfirstlane(wave_max(qlen));
    uint32_t *zw = z ? z + (int64_t)(tid >> 6) * zstride : nullptr;

    // query codes, 8 per VGPR as nibbles in order {c0, c2, c4, c6 | c1, c3, c5, c7} by byte
    // (glob_group splits them into two v_perm selectors)
    // Aligned dword loads (a dword holding a byte of the query never leaves that byte's page),
    // realigned by v_alignbyte; positions >= qlen read as code 4; codes kept to 3 bits.
    uint32_t q8[NG];
    {
        const uintptr_t qa = (uintptr_t)(qer + (live ? p.idq : 0));
        const uint32_t *wp = (const uint32_t *)(qa & ~(uintptr_t)3);
        const int sh = (int)(qa & 3);
        const int nw = (live && qlen > 0) ? (sh + qlen + 3) >> 2 : 0;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            uint32_t wv[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) wv[k] = nw > 0 ? wp[min(2 * g + k, nw - 1)] : 0u;
            uint32_t c0 = __builtin_amdgcn_alignbyte(wv[1], wv[0], sh);
            uint32_t c1 = __builtin_amdgcn_alignbyte(wv[2], wv[1], sh);
            // bytes k >= qlen - 8g -> 4
            const int lim = min(max(qlen - 8 * g, 0), 8);
            const uint64_t m = lim >= 8 ? ~0ull : ((1ull << (8 * lim)) - 1);
            const uint32_t m0 = (uint32_t)m, m1 = (uint32_t)(m >> 32);
            c0 = ((c0 & 0x07070707u) & m0) | (0x04040404u & ~m0);
            c1 = ((c1 & 0x07070707u) & m1) | (0x04040404u & ~m1);
            const uint32_t y0 = (c0 | (c0 >> 4)) & 0x00ff00ffu, y1 = (c1 | (c1 >> 4)) & 0x00ff00ffu;
            q8[g] = __builtin_amdgcn_perm(y1, y0, 0x06040200u);      // {k0|k1<<4, k2|k3<<4, k4|k5<<4, k6|k7<<4}
        }
    }
    // first row: eh[0] = {0, -inf}, eh[j] = {-(o_ins + e_ins j), -inf} for 1 <= j <= min(qlen, w)
    uint32_t R[QMAX];
#pragma unroll
    for (int j = 0; j < QMAX; ++j) {
        const int h = j == 0 ? 0 : ((j <= w && j <= qlen) ? -(gp.o_ins + gp.e_ins * j) : kGNeg);
        R[j] = ((uint32_t)h & 0xffffu) | ((uint32_t)kGNeg << 16);
    }
    int score = qlen == 0 ? 0 : (qlen <= w ? -(gp.o_ins + gp.e_ins * qlen) : kGMinusInf);
    // Narrow traceback window (tb_dw > 0): the path from (0, 0) to (tlen - 1, qlen - 1) runs along the
    // diagonals between 0 and qlen - tlen; each row keeps only the tb_dw dwords from column
    // i + min(0, qlen - tlen) - xs, xs the widest slack whose corridor (|qlen - tlen| + 2 xs + 1
    // columns, any alignment) fits them.  A job with no room (xs < 0) or whose path leaves the
    // corridor goes to retry (the host reruns it with the full band window).  ~3x fewer matrix bytes.
    const int dlt = qlen - tlen;
    const int xs = tb_dw > 0 ? (8 * tb_dw - 8 - abs(dlt)) / 2 : 0;
    const int doff = min(0, dlt) - xs;
    const int rowdw = tb_dw > 0 ? tb_dw : cap_dw;
    const GCx cx{gp.e_del, gp.oe_del, gp.e_ins, gp.oe_ins};
    unsigned long long ncell = 0;
    uint32_t tnext = (live && tlen > 0) ? ref[p.idr] : 4u;
    for (int i = 0; i < tmax; ++i) {
        const bool act = live && i < tlen;
        const uint32_t t = min(tnext, 7u);
        if (act && i + 1 < tlen) tnext = ref[p.idr + i + 1];
        uint2 pr = make_uint2(gp.prof[4][0], gp.prof[4][1]);
        pr = (t == 3) ? make_uint2(gp.prof[3][0], gp.prof[3][1]) : pr;
        pr = (t == 2) ? make_uint2(gp.prof[2][0], gp.prof[2][1]) : pr;
        pr = (t == 1) ? make_uint2(gp.prof[1][0], gp.prof[1][1]) : pr;
        pr = (t == 0) ? make_uint2(gp.prof[0][0], gp.prof[0][1]) : pr;
        const int beg = act ? max(i - w, 0) : 0, end = act ? min(i + w + 1, qlen) : 0;
        GRow r;
        r.lo = max(i - wmax, 0);
        r.hi = min(qmw, i + wmax + 2);
        r.fb = __builtin_amdgcn_readfirstlane(wave_max(act ? beg : 0));
        r.fe = __builtin_amdgcn_readfirstlane(wave_min(act ? end : INT_MAX));
        r.dlo = r.lo >> 3;
        r.cap_dw = cap_dw;
        r.tb_dw = tb_dw;
        const int bnd = -(gp.o_del + gp.e_del * (i + 1));
        int h1 = (act && beg == 0) ? bnd : kGNeg;
        int f = kGNeg;
        glob_row<QMAX>(std::make_integer_sequence<int, NG>{}, R, q8, pr, h1, f, cx, beg, end, r,
                       zw ? zw + (int64_t)i * rowdw * 64 : nullptr, lane, max(i + doff, 0) >> 3);
        if (act) {
            ncell += (unsigned long long)max(end - beg, 0);
            if (end == qlen) score = beg < end ? h1 : (beg == 0 ? bnd : kGMinusInf);
        }
    }
    for (int o = 32; o > 0; o >>= 1) ncell += __shfl_xor(ncell, o);
    if (lane == 0 && cells) atomicAdd(cells, ncell);
    if (!live) return;
    pairs[idx].score = score;
    if (!zw) return;
    if (tb_dw > 0 && xs < 0 && !(qlen >= 1 && tlen >= 1 && qlen < tlen - w)) {
        retry[1 + atomicAdd(retry, 1)] = idx;               // corridor wider than the window
        n_cigar[idx] = -3;
        return;
    }
    glob_traceback(zw, cap_dw, wmax, lane, qlen, tlen, w, cigar + (int64_t)idx * stride, stride, n_cigar + idx,
                   tb_dw, doff, retry, idx);
}

// ------------------------------------------------------------------ band-coordinate kernel
// Slot s of row i holds column j = i - w + s (w = the lane's band), so the band is a fixed
// window of 2w + 1 slots: the diagonal H(i-1, j-1) sits in the SAME slot, E(i, j) was written
// into slot s by the cell of slot s + 1 one row earlier, and the query codes shift one nibble
// per row.  H and E live in separate int32 register arrays (upstream's int32 values and
// MINUS_INF, no packing); the per-row bounds are per-wave scalars computed from wmin / wmax /
// min and max of qlen + w, with no cross-lane reduction in the row loop.
template <bool MASKED>
__device__ __forceinline__ uint32_t glob_bcell(int &H, int &Ecur, int *Eprev, int sc, int &h1, int &f,
                                               const GCx &c, bool in, bool atend, bool lb, int bnd)
{
    const int m = H + sc, e = Ecur;
    int h = max(m, e);
    uint32_t d = m < e ? 1u : 0u;
    d = h < f ? 2u : d;
    h = max(h, f);
    const int t = m - c.oe_del, ee = e - c.e_del;
    const uint32_t eb = ee > t ? 4u : 0u;
    const int e2 = max(ee, t);
    const int t2 = m - c.oe_ins, ff = f - c.e_ins;
    const uint32_t fb = ff > t2 ? 8u : 0u;
    const int f2 = max(ff, t2);
    if (!MASKED) {
        H = h;
        if (Eprev) *Eprev = e2;
        h1 = h; f = f2;
    } else {
        H = in ? h : (lb ? bnd : H);
        if (Eprev) *Eprev = in ? e2 : (atend ? kGMinusInf : *Eprev);
        h1 = in ? h : h1;
        f = in ? f2 : f;
    }
    return d | eb | fb;
}

struct GBand {                      // per-lane slot bounds of a row
    int sb, se, bnd;                // valid slots [sb, se); slot se takes E = -inf; slot sb - 1 (when
    bool left;                      //   the band touches column 0) takes H(i, -1) = bnd
};

template <int G, int BW, bool MASKED>
__device__ __forceinline__ uint32_t glob_bgroup(int (&H)[BW], int (&E)[BW], const uint32_t (&Qb)[BW / 8], uint2 pr,
                                                int &h1, int &f, const GCx &c, const GBand &b)
{
    const uint32_t sel0 = Qb[G] & 0x0f0f0f0fu, sel1 = (Qb[G] >> 4) & 0x0f0f0f0fu;
    const uint32_t pw0 = __builtin_amdgcn_perm(pr.y, pr.x, sel0), pw1 = __builtin_amdgcn_perm(pr.y, pr.x, sel1);
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int s = 8 * G + k;
        const int sc = (int)(int8_t)(((k & 1) ? pw1 : pw0) >> (8 * (k >> 1)));
        const bool in = MASKED ? (s >= b.sb && s < b.se) : true;
        const bool atend = MASKED ? (s == b.se) : false;
        const bool lb = MASKED ? (b.left && s == b.sb - 1) : false;
        word |= glob_bcell<MASKED>(H[s], E[s], s > 0 ? &E[s - 1] : nullptr, sc, h1, f, c, in, atend, lb, b.bnd)
                << (4 * k);
    }
    return word;
}

template <int G, int BW>
__device__ __forceinline__ void glob_bgroup_at(int (&H)[BW], int (&E)[BW], const uint32_t (&Qb)[BW / 8], uint2 pr,
                                               int &h1, int &f, const GCx &c, const GBand &b, int lo, int hi, int fb,
                                               int fe, uint32_t *__restrict__ zrow, int lane)
{
    if (8 * G + 8 <= lo || 8 * G >= hi) return;          // uniform
    uint32_t word;
    if (8 * G >= fb && 8 * G + 8 <= fe) word = glob_bgroup<G, BW, false>(H, E, Qb, pr, h1, f, c, b);
    else word = glob_bgroup<G, BW, true>(H, E, Qb, pr, h1, f, c, b);
    if (zrow) zrow[G * 64 + lane] = word;
}

template <int BW, int... G>
__device__ __forceinline__ void glob_brow(std::integer_sequence<int, G...>, int (&H)[BW], int (&E)[BW],
                                          const uint32_t (&Qb)[BW / 8], uint2 pr, int &h1, int &f, const GCx &c,
                                          const GBand &b, int lo, int hi, int fb, int fe, uint32_t *__restrict__ zrow,
                                          int lane)
{
    (glob_bgroup_at<G, BW>(H, E, Qb, pr, h1, f, c, b, lo, hi, fb, fe, zrow, lane), ...);
}

// traceback over band-coordinate nibbles: cell (i, k) sits in slot k - i + w
__device__ void glob_traceback_band(const uint32_t *__restrict__ zw, int ng, int lane, int qlen, int tlen, int w,
                                    uint32_t *__restrict__ out, int stride, int32_t *__restrict__ nout)
{
    if (qlen >= 1 && tlen >= 1 && qlen < tlen - w) { *nout = -2; return; }
    int i = tlen - 1, k = min(i + w + 1, qlen) - 1, which = 0, n = 0;
    uint32_t cur = 0;
    auto push = [&](uint32_t op, uint32_t len) {
        if (n > 0 && (cur & 0xfu) == op) { cur += len << 4; return; }
        if (n > 0 && n - 1 < stride) out[n - 1] = cur;
        cur = len << 4 | op;
        ++n;
    };
    while (i >= 0 && k >= 0) {
        const int s = k - i + w;
        const uint32_t word = zw[((int64_t)i * ng + (s >> 3)) * 64 + lane];
        const uint32_t nib = (word >> ((s & 7) * 4)) & 15u;
        which = which == 0 ? (int)(nib & 3u) : which == 1 ? (int)((nib >> 2) & 1u) : ((nib & 8u) ? 2 : 0);
        if (which == 0) { push(0, 1); --i; --k; }
        else if (which == 1) { push(2, 1); --i; }
        else { push(1, 1); --k; }
    }
    if (i >= 0) push(2, (uint32_t)(i + 1));
    if (k >= 0) push(1, (uint32_t)(k + 1));
    if (n > 0 && n - 1 < stride) out[n - 1] = cur;
    if (n > stride) { *nout = -1; return; }
    for (int a = 0, b = n - 1; a < b; ++a, --b) {
        const uint32_t t = out[a];
        out[a] = out[b];
        out[b] = t;
    }
    *nout = n;
}

template <int BW>
__global__ __launch_bounds__(64, 2) void glob_band_kernel(
    const GlobParams gp, SeqPair *__restrict__ pairs, const int32_t *__restrict__ order, int32_t n,
    const uint8_t *__restrict__ ref, const uint8_t *__restrict__ qer, uint32_t *__restrict__ z, int64_t zstride,
    uint32_t *__restrict__ cigar, int32_t stride, int32_t *__restrict__ n_cigar, unsigned long long *__restrict__ cells)
{
    constexpr int NG = BW / 8;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool live = tid < n;
    const int idx = live ? order[tid] : 0;
    SeqPair p{};
    if (live) p = pairs[idx];
    const int qlen = live ? p.len2 : 0, tlen = live ? p.len1 : 0, w = live ? p.h0 : 0;
    const int wmax = __builtin_amdgcn_readfirstlane(wave_max(live ? w : -1));
    if (wmax < 0) return;                                   // whole wave empty
    const int wmin = __builtin_amdgcn_readfirstlane(wave_min(live ? w : INT_MAX));
    const int tmax = __builtin_amdgcn_readfirstlane(wave_max(tlen));
    const int qwmin = __builtin_amdgcn_readfirstlane(wave_min(live ? qlen + w : INT_MAX));
    const int qwmax = __builtin_amdgcn_readfirstlane(wave_max(live ? qlen + w : 0));
    uint32_t *zw = z ? z + (int64_t)(tid >> 6) * zstride : nullptr;
    const uint8_t *q = qer + p.idq;
    // query codes of row 0 in band coordinates: slot s <-> column s - w, 8 nibbles per dword
    uint32_t Qb[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        uint32_t w8 = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = 8 * g + k - w;
            const uint32_t code = (live && j >= 0 && j < qlen) ? q[j] : 4u;
            w8 |= min(code, 7u) << (4 * k);
        }
        Qb[g] = w8;
    }
    // row -1: H(-1, j - 1) = eh[j].h of upstream's first row, E(0, j) = -inf
    int H[BW], E[BW];
#pragma unroll
    for (int s = 0; s < BW; ++s) {
        const int j = s - w;
        H[s] = j == 0 ? 0 : ((j >= 1 && j <= w && j <= qlen) ? -(gp.o_ins + gp.e_ins * j) : kGMinusInf);
        E[s] = kGMinusInf;
    }
    int score = qlen == 0 ? 0 : (qlen <= w ? -(gp.o_ins + gp.e_ins * qlen) : kGMinusInf);
    const GCx cx{gp.e_del, gp.oe_del, gp.e_ins, gp.oe_ins};
    unsigned long long ncell = 0;
    uint32_t tnext = (live && tlen > 0) ? ref[p.idr] : 4u;
    int jn = BW - w;                                        // column entering the top slot next row
    uint32_t qnext = (live && jn >= 0 && jn < qlen) ? q[jn] : 4u;
    for (int i = 0; i < tmax; ++i) {
        const bool act = live && i < tlen;
        const uint32_t t = min(tnext, 7u);
        if (act && i + 1 < tlen) tnext = ref[p.idr + i + 1];
        uint2 pr = make_uint2(gp.prof[4][0], gp.prof[4][1]);
        pr = (t == 3) ? make_uint2(gp.prof[3][0], gp.prof[3][1]) : pr;
        pr = (t == 2) ? make_uint2(gp.prof[2][0], gp.prof[2][1]) : pr;
        pr = (t == 1) ? make_uint2(gp.prof[1][0], gp.prof[1][1]) : pr;
        pr = (t == 0) ? make_uint2(gp.prof[0][0], gp.prof[0][1]) : pr;
        const int beg = max(i - w, 0), end = min(i + w + 1, qlen);
        GBand b;
        b.sb = act ? beg - i + w : BW + 1;
        b.se = act ? end - i + w : -1;
        b.bnd = -(gp.o_del + gp.e_del * (i + 1));
        b.left = act && beg == 0;
        // uniform bounds: slots any lane touches [lo, hi) (incl. the boundary slot sb - 1 and the
        // end slot se), slots every active lane has in band [fb, fe)
        const int lo = max(wmin - i - 1, 0);
        const int hi = min(BW, min(2 * wmax + 1, qwmax - i) + 1);
        const int fb = max(wmax - i, 0);
        const int fe = min(2 * wmin + 1, qwmin - i);
        int h1 = b.left ? b.bnd : kGMinusInf;
        int f = kGMinusInf;
        glob_brow<BW>(std::make_integer_sequence<int, NG>{}, H, E, Qb, pr, h1, f, cx, b, lo, hi, fb, fe,
                      zw ? zw + (int64_t)i * NG * 64 : nullptr, lane);
        if (act) {
            ncell += (unsigned long long)max(end - beg, 0);
            if (end == qlen) score = beg < end ? h1 : (beg == 0 ? b.bnd : kGMinusInf);
        }
        // next row's query window: shift one slot (nibble) down, the new top slot from qnext
#pragma unroll
        for (int g = 0; g < NG - 1; ++g) Qb[g] = __builtin_amdgcn_alignbit(Qb[g + 1], Qb[g], 4);
        Qb[NG - 1] = (Qb[NG - 1] >> 4) | (min(qnext, 7u) << 28);
        ++jn;
        qnext = (live && jn >= 0 && jn < qlen) ? q[jn] : 4u;
    }
    for (int o = 32; o > 0; o >>= 1) ncell += __shfl_xor(ncell, o);
    if (lane == 0 && cells) atomicAdd(cells, ncell);
    if (!live) return;
    pairs[idx].score = score;
    if (zw) glob_traceback_band(zw, NG, lane, qlen, tlen, w, cigar + (int64_t)idx * stride, stride, n_cigar + idx);
}

// ------------------------------------------------------------------ wide kernel
__global__ __launch_bounds__(256) void glob_wide_kernel(
    const GlobParams gp, SeqPair *__restrict__ pairs, const int32_t *__restrict__ order, int32_t n,
    const uint8_t *__restrict__ ref, const uint8_t *__restrict__ qer, uint32_t *__restrict__ z, int64_t zstride,
    int32_t cap_dw, int2 *__restrict__ ehs, uint32_t *__restrict__ cigar, int32_t stride,
    int32_t *__restrict__ n_cigar, unsigned long long *__restrict__ cells)
{
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool live = tid < n;
    const int idx = live ? order[tid] : 0;
    SeqPair p{};
    if (live) p = pairs[idx];
    const int wmax = __builtin_amdgcn_readfirstlane(wave_max(live ? p.h0 : -1));
    unsigned long long ncell = 0;
    int score = 0;
    uint32_t *zw = (z && wmax >= 0) ? z + (int64_t)(tid >> 6) * zstride : nullptr;
    if (live) {
        const int qlen = p.len2, tlen = p.len1, w = p.h0;
        const uint8_t *query = qer + p.idq, *target = ref + p.idr;
#define EH(j) ehs[(int64_t)(j) * n + tid]
        EH(0) = make_int2(0, kGMinusInf);
        int j = 1;
        for (; j <= qlen && j <= w; ++j) EH(j) = make_int2(-(gp.o_ins + gp.e_ins * j), kGMinusInf);
        for (; j <= qlen; ++j) EH(j) = make_int2(kGMinusInf, kGMinusInf);
        for (int i = 0; i < tlen; ++i) {
            int f = kGMinusInf;
            const int8_t *row = gp.mat + 5 * min((int)target[i], 4);
            const int beg = i > w ? i - w : 0;
            const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
            int h1 = beg == 0 ? -(gp.o_del + gp.e_del * (i + 1)) : kGMinusInf;
            const int dlo = max(i - wmax, 0) >> 3;
            uint32_t *zrow = zw ? zw + (int64_t)i * cap_dw * 64 : nullptr;
            uint32_t word = 0;
            int dcur = beg >> 3;
            for (j = beg; j < end; ++j) {
                int2 q = EH(j);
                int mm = q.x + row[min((int)query[j], 4)], e = q.y, h;
                q.x = h1;
                uint32_t d = mm >= e ? 0u : 1u;
                h = mm >= e ? mm : e;
                d = h >= f ? d : 2u;
                h = h >= f ? h : f;
                h1 = h;
                int t = mm - gp.oe_del;
                e -= gp.e_del;
                d |= e > t ? 4u : 0u;
                e = e > t ? e : t;
                q.y = e;
                EH(j) = q;
                t = mm - gp.oe_ins;
                f -= gp.e_ins;
                d |= f > t ? 8u : 0u;
                f = f > t ? f : t;
                if ((j >> 3) != dcur) {
                    if (zrow) zrow[(dcur - dlo) * 64 + lane] = word;
                    dcur = j >> 3;
                    word = 0;
                }
                word |= d << ((j & 7) * 4);
            }
            if (zrow && beg < end) zrow[(dcur - dlo) * 64 + lane] = word;
            EH(end) = make_int2(h1, kGMinusInf);
            ncell += (unsigned long long)max(end - beg, 0);
        }
        score = EH(qlen).x;
#undef EH
    }
    if (wmax >= 0) {
        for (int o = 32; o > 0; o >>= 1) ncell += __shfl_xor(ncell, o);
        if (lane == 0 && cells) atomicAdd(cells, ncell);
    }
    if (!live) return;
    pairs[idx].score = score;
    if (zw) glob_traceback(zw, cap_dw, wmax, lane, p.len2, p.len1, p.h0, cigar + (int64_t)idx * stride, stride,
                           n_cigar + idx);
}

// ------------------------------------------------------------------ launchers
hipError_t launch_glob_plan(const SeqPair *pairs, int32_t n, const GlobParams &gp, uint32_t *keys,
                            int32_t *vals, int32_t *meta, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(meta, 0, sizeof(int32_t) * kGMetaWords, s);   // all slots
    if (e != hipSuccess || n <= 0) return e;
    hipLaunchKernelGGL(glob_plan_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, pairs, n, gp, keys,
                       vals, meta);
    return hipGetLastError();
}

template <int QMAX>
static void launch_lane_q(const GlobParams &gp, SeqPair *pairs, const int32_t *order, int32_t n,
                          const uint8_t *ref, const uint8_t *qer, uint32_t *z, int64_t zstride, int32_t cap_dw,
                          uint32_t *cigar, int32_t stride, int32_t *n_cigar, unsigned long long *cells,
                          hipStream_t s, int32_t tb_dw, int32_t *retry)
{
    hipLaunchKernelGGL(glob_lane_kernel<QMAX>, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, gp, pairs,
                       order, n, ref, qer, z, zstride, cap_dw, cigar, stride, n_cigar, cells, tb_dw, retry);
}

hipError_t launch_glob_class(int cls, const GlobParams &gp, SeqPair *pairs, const int32_t *order, int32_t n,
                             const uint8_t *ref, const uint8_t *qer, uint32_t *z, int64_t zstride,
                             int32_t cap_dw, int2 *ehs, uint32_t *cigar, int32_t stride, int32_t *n_cigar,
                             unsigned long long *cells, hipStream_t s, int32_t tb_dw, int32_t *retry)
{
    if (n <= 0) return hipSuccess;
    if (tb_dw > 0 && (!retry || !z || cls < kGlobLane0 || cls >= kGlobWideClass)) return hipErrorInvalidValue;
    switch (cls) {
#define GB(C, BW)                                                                                           \
    case C:                                                                                                 \
        hipLaunchKernelGGL(glob_band_kernel<BW>, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, gp, pairs,    \
                           order, n, ref, qer, z, zstride, cigar, stride, n_cigar, cells);                 \
        break;
    GB(0, 32) GB(1, 48) GB(2, 64) GB(3, 80) GB(4, 96)
#undef GB
    case kGlobLane0 + 0: launch_lane_q<32>(gp, pairs, order, n, ref, qer, z, zstride, cap_dw, cigar, stride, n_cigar, cells, s, tb_dw, retry); break;
    case kGlobLane0 + 1: launch_lane_q<64>(gp, pairs, order, n, ref, qer, z, zstride, cap_dw, cigar, stride, n_cigar, cells, s, tb_dw, retry); break;
    case kGlobLane0 + 2: launch_lane_q<96>(gp, pairs, order, n, ref, qer, z, zstride, cap_dw, cigar, stride, n_cigar, cells, s, tb_dw, retry); break;
    case kGlobLane0 + 3: launch_lane_q<128>(gp, pairs, order, n, ref, qer, z, zstride, cap_dw, cigar, stride, n_cigar, cells, s, tb_dw, retry); break;
    case kGlobLane0 + 4: launch_lane_q<160>(gp, pairs, order, n, ref, qer, z, zstride, cap_dw, cigar, stride, n_cigar, cells, s, tb_dw, retry); break;
    case kGlobWideClass:
        hipLaunchKernelGGL(glob_wide_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, gp, pairs, order,
                           n, ref, qer, z, zstride, cap_dw, ehs, cigar, stride, n_cigar, cells);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace bsw
