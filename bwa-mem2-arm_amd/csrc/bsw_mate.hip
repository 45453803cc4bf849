// bsw_mate.hip -- CDNA4 (gfx950) batch kernel for mate rescue: local Smith-Waterman with
// upstream ksw_align2 / ksw_u8 / ksw_i16 semantics (include/bsw_mate.h, SURVEY.md §8(f) row 2,
// DESIGN.md §4.9).
//
// Layout: one LANE per job, the whole DP row of the job in VGPRs as packed {h:16, e:16}
// per query column (the lane kernel's layout, bsw_kernels.hip), query codes 4 per VGPR,
// scores from a per-row 8-byte profile by v_perm.  Full-width rows (no band), ncol = slen * P
// columns where upstream's striped kernels use slen = ceil(qlen / P) vectors of P lanes
// (P = 16 for u8, 8 for i16) and pad the query with score-0 positions.
//
// Upstream's result depends on the striping in one place: E(i+1, j) is computed from H
// before the lazy-F loop propagates F across the P segment boundaries (j = k * slen).  In
// query order that is two F chains (tests/ksw_align_py.py is the same formulation in Python):
//   f  -- in-segment F, reset to 0 entering a segment start; feeds H1, E and itself;
//   fx -- cross-segment F (what the lazy-F loop carries), fed by f at segment starts,
//         decays by e_ins; feeds only the H the next row sees: H = max(H1, fx).
// Row maximum and the query end qe come from H1 (upstream's row max is taken before lazy-F;
// fx < row max when o_ins >= 1, so the argmax positions agree).  Segment starts are
// wave-uniform: the host sorts jobs into buckets of equal (P, slen), each padded to whole
// waves, so the boundary test is a scalar bit test per column.
//
// Secondary hits (KSW_XSUBO): each row's maximum is stored to an HBM scratch laid out
// [row][slot] (coalesced per wavefront) and replayed per lane after the last row through
// upstream's b-array rule, once te and the score -- hence the exclusion window -- are known.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include <utility>
#include "bsw_mate_k.h"
#include "bsw_wave.h"

namespace bsw {

__device__ __forceinline__ int mmax3(int a, int b, int c) { return max(max(a, b), c); }

// (P, slen) bucket of a job; -1: no job.  Buckets 0..16: u8 (slen 0..16), 17..49: i16 (0..32).
__device__ __forceinline__ int mate_bucket(int qlen, int xtra)
{
    const bool u8 = (xtra & BSW_KSW_XBYTE) != 0;
    const int P = u8 ? 16 : 8;
    const int L = (qlen + P - 1) / P;
    return u8 ? L : 17 + L;
}

__host__ __device__ __forceinline__ int mate_bucket_ncol(int b) { return b <= 16 ? 16 * b : 8 * (b - 17); }

// Reverse-pass geometry (ksw_align2's second call): query = reverse(query[0, qe]), target =
// reverse(target[0, te]) then target[te+1, tlen) unchanged, xtra = KSW_XSTOP | score.
__device__ __forceinline__ bool mate_rev_needed(int xtra, const bsw_kswr_t &r)
{
    if (!(xtra & BSW_KSW_XSTART)) return false;
    return !((xtra & BSW_KSW_XSUBO) && r.score < (xtra & 0xffff));
}

__global__ void mate_count_kernel(const SeqPair *__restrict__ pairs, const bsw_kswr_t *__restrict__ aln,
                                  int32_t n, int mode, int32_t *__restrict__ meta)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int b = -1, tl = 0;
    if (i < n) {
        const SeqPair p = pairs[i];
        if (mode == 0) {
            if (p.len2 < 0 || p.len2 > BSW_MATE_MAX_QLEN || p.len1 < 0 || p.len1 > BSW_MAX_LEN) {
                atomicOr(&meta[kMateMetaErr], 1);
            } else {
                b = mate_bucket(p.len2, p.h0);
                tl = p.len1;
            }
        } else if (mate_rev_needed(p.h0, aln[i])) {
            b = mate_bucket(aln[i].qe + 1, p.h0);
            tl = p.len1;
        }
    }
    const int lane = threadIdx.x & 63;
    const int tmax = wave_max(tl);
    if (lane == 0 && tmax > 0) atomicMax(&meta[kMateMetaTmax], tmax);
    unsigned long long pending = __ballot(b >= 0);
    while (pending) {                                   // one atomic per (wave, bucket)
        const int leader = __ffsll((long long)pending) - 1;
        const int bl = __shfl(b, leader);
        const unsigned long long m = __ballot(b == bl);
        if (lane == leader) atomicAdd(&meta[kMateMetaCount + bl], __popcll(m));
        pending &= ~m;
    }
}

// One thread: bucket starts in ncol-class order, each bucket padded to whole waves.
__global__ void mate_offsets_kernel(int32_t *__restrict__ meta)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int pos = 0;
    for (int c = 0; c < kMateClasses; ++c) {
        meta[kMateMetaClass + 2 * c] = pos;
        for (int b = 0; b < kMateBuckets; ++b) {
            if (mate_class_of_ncol(mate_bucket_ncol(b)) != c) continue;
            meta[kMateMetaCursor + b] = pos;
            pos += (meta[kMateMetaCount + b] + 63) & ~63;
        }
        meta[kMateMetaClass + 2 * c + 1] = pos;
    }
    meta[kMateMetaTotal] = pos;
}

__global__ void mate_scatter_kernel(const SeqPair *__restrict__ pairs, const bsw_kswr_t *__restrict__ aln,
                                    int32_t n, int mode, int32_t *__restrict__ meta,
                                    int32_t *__restrict__ jobs)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int b = -1;
    if (i < n) {
        const SeqPair p = pairs[i];
        if (mode == 0) {
            if (p.len2 >= 0 && p.len2 <= BSW_MATE_MAX_QLEN && p.len1 >= 0 && p.len1 <= BSW_MAX_LEN)
                b = mate_bucket(p.len2, p.h0);
        } else if (mate_rev_needed(p.h0, aln[i])) {
            b = mate_bucket(aln[i].qe + 1, p.h0);
        }
    }
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1ull;
    unsigned long long pending = __ballot(b >= 0);
    while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const int bl = __shfl(b, leader);
        const unsigned long long m = __ballot(b == bl);
        int base = 0;
        if (lane == leader) base = atomicAdd(&meta[kMateMetaCursor + bl], __popcll(m));
        base = __shfl(base, leader);
        if (b == bl) jobs[base + __popcll(m & below)] = i;
        pending &= ~m;
    }
}

struct MateCx {
    int e_del, oe_del, e_ins, oe_ins;
};

// One column J: H1 = max(Hdiag + S, E, f); H = max(H1, fx); E' from H1; f' in-segment.
// eh[J] = { H(i-1, J-1), E(i, J) } in, { H(i, J-1), E(i+1, J) } out.
template <int J>
__device__ __forceinline__ void mate_cell(uint32_t &v, int s, int &f, int &fx, int &hprev, int &key,
                                          const MateCx &c)
{
    const int hd = (int)(v & 0xffffu), e = (int)(v >> 16);
    const int h1 = mmax3(hd + s, e, f);                  // >= 0 (e >= 0)
    const int e2 = mmax3(e - c.e_del, h1 - c.oe_del, 0);
    f = mmax3(f - c.e_ins, h1 - c.oe_ins, 0);
    const int h = max(h1, fx);
    fx -= c.e_ins;
    v = (uint32_t)hprev | ((uint32_t)e2 << 16);
    hprev = h;
    key = max(key, (h1 << 8) | (255 - J));               // row max, ties to the smallest j
}

template <int G, int NC>
__device__ __forceinline__ void mate_group(uint32_t (&eh)[NC], const uint32_t (&q4)[NC / 4], uint2 pr,
                                           const uint32_t (&bm)[(NC + 31) / 32], int ncol, int &f, int &fx,
                                           int &hprev, int &key, const MateCx &c)
{
    if (4 * G >= ncol) return;                           // uniform
    const uint32_t pw = __builtin_amdgcn_perm(pr.y, pr.x, q4[G]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        constexpr int J0 = 4 * G;
        const int J = J0 + k;
        // segment start (wave-uniform bit): the in-segment F chain hands over to fx.  A scalar
        // bit test + branch in asm, so the per-column condition is not hoisted out of the row
        // loop (that would pin two SGPRs per column).
        asm volatile("s_bitcmp1_b32 %[w], %[b]\n\t"
                     "s_cbranch_scc0 1f\n\t"
                     "v_max_i32_e32 %[fx], %[fx], %[f]\n\t"
                     "v_mov_b32_e32 %[f], 0\n"
                     "1:"
                     : [f] "+v"(f), [fx] "+v"(fx)
                     : [w] "s"(bm[J >> 5]), [b] "i"(J & 31)
                     : "scc");
        switch (k) {
        case 0: mate_cell<J0 + 0>(eh[J0 + 0], (int)(int8_t)(pw), f, fx, hprev, key, c); break;
        case 1: mate_cell<J0 + 1>(eh[J0 + 1], (int)(int8_t)(pw >> 8), f, fx, hprev, key, c); break;
        case 2: mate_cell<J0 + 2>(eh[J0 + 2], (int)(int8_t)(pw >> 16), f, fx, hprev, key, c); break;
        default: mate_cell<J0 + 3>(eh[J0 + 3], (int)(int8_t)(pw >> 24), f, fx, hprev, key, c); break;
        }
    }
}

template <int NC, int... G>
__device__ __forceinline__ void mate_row(std::integer_sequence<int, G...>, uint32_t (&eh)[NC],
                                         const uint32_t (&q4)[NC / 4], uint2 pr,
                                         const uint32_t (&bm)[(NC + 31) / 32], int ncol, int &key,
                                         const MateCx &c)
{
    int f = 0, fx = 0, hprev = 0;
    (mate_group<G, NC>(eh, q4, pr, bm, ncol, f, fx, hprev, key, c), ...);
}

template <int NC>
__global__ __launch_bounds__(64, NC <= 160 ? 2 : 1) void mate_kernel(
    const MateParams mp, const SeqPair *__restrict__ pairs, const int32_t *__restrict__ jobs, int32_t j0,
    int32_t j1, const uint8_t *__restrict__ ref, const uint8_t *__restrict__ qer, bsw_kswr_t *__restrict__ aln,
    int mode, uint16_t *__restrict__ scratch, int64_t sstride, unsigned long long *__restrict__ cells)
{
    constexpr int NG = NC / 4, NW = (NC + 31) / 32;
    const int slot = j0 + blockIdx.x * blockDim.x + threadIdx.x;
    const int idx = slot < j1 ? jobs[slot] : -1;
    const bool live = idx >= 0;
    int idr = 0, idq = 0, tlen = 0, qlen = 0, xtra = 0, te0 = -1, qe0 = -1, score0 = 0;
    if (live) {
        const SeqPair p = pairs[idx];
        idr = p.idr; idq = p.idq; tlen = p.len1; qlen = p.len2; xtra = p.h0;
        if (mode == 1) {
            const bsw_kswr_t r = aln[idx];
            te0 = r.te; qe0 = r.qe; score0 = r.score;
            qlen = qe0 + 1;
            xtra = BSW_KSW_XSTOP | (score0 & 0xffff) | (xtra & BSW_KSW_XBYTE);
        }
    }
    const bool u8 = (xtra & BSW_KSW_XBYTE) != 0;
    const int P = u8 ? 16 : 8;
    const int L = (qlen + P - 1) / P;
    const int Lw = __builtin_amdgcn_readfirstlane(wave_max(live ? L : -1));     // uniform by bucketing
    const int ncw = __builtin_amdgcn_readfirstlane(wave_max(live ? L * P : -1));
    if (Lw < 0) return;                                   // whole wave empty (no LDS, no barriers)
    const int minsc = (xtra & BSW_KSW_XSUBO) ? (xtra & 0xffff) : 0x10000;
    const int endsc = (xtra & BSW_KSW_XSTOP) ? (xtra & 0xffff) : 0x10000;

    // query codes (4 per VGPR); positions >= qlen are code 5 (score 0: upstream's padding)
    uint32_t q4[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        uint32_t w4 = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = 4 * g + k;
            uint32_t code = 5;
            if (live && j < qlen) code = mode == 0 ? qer[idq + j] : qer[idq + qe0 - j];
            w4 |= min(code, 7u) << (8 * k);
        }
        q4[g] = w4;
    }
    // segment starts j = k * slen (0 < j < ncol): wave-uniform bit mask
    uint32_t bm[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        uint32_t bits = 0;
        for (int j = (Lw > 0 ? ((32 * w + Lw - 1) / Lw) * Lw : INT_MAX); j < 32 * w + 32 && j < ncw; j += Lw)
            if (j > 0) bits |= 1u << (j - 32 * w);
        bm[w] = __builtin_amdgcn_readfirstlane(bits);
    }
    uint32_t eh[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) eh[j] = 0;
    const MateCx cx{mp.e_del, mp.oe_del, mp.e_ins, mp.oe_ins};

    int gmax = 0, te = -1, qe = (live && L > 0) ? 0 : -1, rows = 0;
    bool run = live && tlen > 0;
    auto row_base = [&](int i) -> int { return (mode == 1 && i <= te0) ? te0 - i : i; };
    uint32_t tnext = run ? ref[idr + row_base(0)] : 0;
    for (int i = 0;; ++i) {
        const bool act = run && i < tlen;
        if (__ballot(act) == 0) break;
        if (act) {
            const uint32_t t = min(tnext, 7u);
            if (i + 1 < tlen) tnext = ref[idr + row_base(i + 1)];
            const uint2 pr = make_uint2(mp.prof[t][0], mp.prof[t][1]);
            int key = 0, ncr;
            // opaque per-row copy of ncol: keeps the per-group bound tests inside the loop
            asm volatile("s_mov_b32 %0, %1" : "=s"(ncr) : "s"(ncw));
            mate_row<NC>(std::make_integer_sequence<int, NG>{}, eh, q4, pr, bm, ncr, key, cx);
            const int imax = key >> 8;
            if (scratch) scratch[(int64_t)i * sstride + slot] = (uint16_t)imax;
            rows = i + 1;
            if (imax > gmax) {
                gmax = imax; te = i; qe = 255 - (key & 255);
                if ((u8 && gmax + mp.shift >= 255) || gmax >= endsc) run = false;
            }
        } else {
            run = false;
        }
    }
    // DP cells actually run (statistics)
    {
        unsigned long long cl = live ? (unsigned long long)rows * (unsigned long long)(L * P) : 0ull;
        for (int o = 32; o > 0; o >>= 1) cl += __shfl_xor(cl, o);
        if ((threadIdx.x & 63) == 0 && cells) atomicAdd(cells, cl);
    }
    if (!live) return;
    const bool sat = u8 && gmax + mp.shift >= 255;
    const int score = sat ? 255 : gmax;
    if (mode == 1) {
        if (score == score0) { aln[idx].tb = te0 - te; aln[idx].qb = qe0 - qe; }
        return;
    }
    bsw_kswr_t r;
    r.score = score; r.te = te; r.qe = -1; r.score2 = -1; r.te2 = -1; r.tb = -1; r.qb = -1;
    if (!sat) {
        r.qe = qe;
        if (minsc <= 0xffff && scratch) {                 // upstream's b array, replayed
            const int wdw = (score + mp.maxsc - 1) / mp.maxsc;
            const int low = te - wdw, high = te + wdw;
            int cur_sc = 0, cur_row = -2;
            bool have = false;
            auto consider = [&](int sc, int row) {
                if ((row < low || row > high) && sc > r.score2) { r.score2 = sc; r.te2 = row; }
            };
            for (int i = 0; i < rows; ++i) {
                const int im = scratch[(int64_t)i * sstride + slot];
                if (im < minsc) continue;
                if (!have || cur_row + 1 != i) {
                    if (have) consider(cur_sc, cur_row);
                    have = true; cur_sc = im; cur_row = i;
                } else if (cur_sc < im) {
                    cur_sc = im; cur_row = i;
                }
            }
            if (have) consider(cur_sc, cur_row);
        }
    }
    aln[idx] = r;
}

template <int NC>
static hipError_t launch_nc(const MateParams &mp, const SeqPair *pairs, const int32_t *jobs, int32_t j0,
                            int32_t j1, const uint8_t *ref, const uint8_t *qer, bsw_kswr_t *aln, int mode,
                            uint16_t *scratch, int64_t sstride, unsigned long long *cells, hipStream_t s)
{
    const int n = j1 - j0;
    hipLaunchKernelGGL(mate_kernel<NC>, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, mp, pairs, jobs,
                       j0, j1, ref, qer, aln, mode, scratch, sstride, cells);
    return hipGetLastError();
}

hipError_t launch_mate_prepare(const SeqPair *pairs, const bsw_kswr_t *aln, int32_t n, int mode,
                               int32_t *meta, int32_t *jobs, int32_t jobs_cap, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(meta, 0, sizeof(int32_t) * kMateMetaWords, s);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(jobs, 0xff, sizeof(int32_t) * (size_t)jobs_cap, s)) != hipSuccess) return e;
    const unsigned nb = (unsigned)((n + 255) / 256);
    if (n > 0) hipLaunchKernelGGL(mate_count_kernel, dim3(nb), dim3(256), 0, s, pairs, aln, n, mode, meta);
    hipLaunchKernelGGL(mate_offsets_kernel, dim3(1), dim3(64), 0, s, meta);
    if (n > 0) hipLaunchKernelGGL(mate_scatter_kernel, dim3(nb), dim3(256), 0, s, pairs, aln, n, mode, meta, jobs);
    return hipGetLastError();
}

hipError_t launch_mate_class(int cls, const MateParams &mp, const SeqPair *pairs, const int32_t *jobs,
                             int32_t j0, int32_t j1, const uint8_t *ref, const uint8_t *qer, bsw_kswr_t *aln,
                             int mode, uint16_t *scratch, int64_t sstride, unsigned long long *cells,
                             hipStream_t s)
{
    if (j1 <= j0) return hipSuccess;
    switch (kMateNcol[cls]) {
    case 64: return launch_nc<64>(mp, pairs, jobs, j0, j1, ref, qer, aln, mode, scratch, sstride, cells, s);
    case 128: return launch_nc<128>(mp, pairs, jobs, j0, j1, ref, qer, aln, mode, scratch, sstride, cells, s);
    case 160: return launch_nc<160>(mp, pairs, jobs, j0, j1, ref, qer, aln, mode, scratch, sstride, cells, s);
    case 192: return launch_nc<192>(mp, pairs, jobs, j0, j1, ref, qer, aln, mode, scratch, sstride, cells, s);
    case 256: return launch_nc<256>(mp, pairs, jobs, j0, j1, ref, qer, aln, mode, scratch, sstride, cells, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace bsw
