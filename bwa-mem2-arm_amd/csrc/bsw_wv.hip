// bsw_wv.hip -- wave-per-alignment band kernel for long queries (gfx950).
//
// The lane kernels (bsw_pc.hip, bsw_kernels.hip) keep one pair's whole DP row in one lane's
// VGPRs, which caps the query at 160 columns.  Here ONE WAVEFRONT runs ONE SeqPair: the row
// is spread over the 64 lanes, C columns per lane, as a window of 64*C absolute columns that
// slides right with the band ([beg, end) never spans more than 2*w + 2 columns, so queries
// of any length up to kWvQmax run in registers as long as 2*wl + C + 2 <= 64*C).
//
// Per row i (ksw_extend2, SURVEY.md Appendix A.4, exact):
//   column-independent work, two columns per v_pk_* instruction:
//     M = hold + min(S, hold)           (the A.5 gate; max(mat) == 1)
//     E' = max(E - e_del, M - oe_del),  ME = max(M, E)       (E, T unclamped as in bsw_pc.hip)
//   the F chain as a prefix maximum (a wave scan instead of a serial walk over columns):
//     F(j) = max(0, P(j) - (j-1) e_ins),  P(j) = max_{beg <= k < j} (M(k) - oe_ins + k e_ins)
//     (F(beg) = 0 and F(j+1) = max(F(j) - e, max(M(j) - oe, 0)) unrolled), P by a lane-local
//     prefix over C columns + a DPP max scan over the 64 lanes;
//   H = max(ME, F); hold(j) <- H(i, j-1) (a one-column shift, lane to lane by DPP);
//   writes limited to slots <= end (slots > end keep their stale values, A.7), E(end) = 0;
//   row max and its LAST column by a 32-bit key (H << 16 | j) max-reduced over the wave;
//   end_{i+1} = min(lastH + 3, qlen) from the last positive H.
// Everything else (z-drop, gscore at end == qlen, max_off, band cap) is wave-uniform scalar
// code.  Scores: per row one LDS read of the target base's 8-byte profile (uniform), per
// 4 columns one v_perm over the lane's query codes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include "bsw_kernels.h"
#include "bsw_wave.h"

namespace bsw {

namespace {

constexpr int kWvNeg = -30000;                 // "-inf" of the F prefix (int16 lanes)

__device__ __forceinline__ uint32_t pk2(int v) { return ((uint32_t)v & 0xffffu) * 0x10001u; }

#define WV_OP2(name, ins)                                                                    \
    __device__ __forceinline__ uint32_t name(uint32_t a, uint32_t b)                        \
    {                                                                                        \
        uint32_t d;                                                                          \
        asm(ins " %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));                                   \
        return d;                                                                            \
    }
WV_OP2(pmax, "v_pk_max_i16")
WV_OP2(pmin, "v_pk_min_i16")
WV_OP2(padd, "v_pk_add_u16")
WV_OP2(psub, "v_pk_sub_i16")
#undef WV_OP2

// {a.lo, max(a.lo, a.hi)}: two-column inclusive prefix inside one register
__device__ __forceinline__ uint32_t ppre(uint32_t a)
{
    uint32_t d;
    asm("v_pk_max_i16 %0, %1, %1 op_sel:[0,0] op_sel_hi:[0,1]" : "=v"(d) : "v"(a));
    return d;
}
// max(a, {b.hi, b.hi})
__device__ __forceinline__ uint32_t pmax_bhi(uint32_t a, uint32_t b)
{
    uint32_t d;
    asm("v_pk_max_i16 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
// packed lanes where a < b (signed 16-bit) -> 0xffff
__device__ __forceinline__ uint32_t plt(uint32_t a, uint32_t b)
{
    uint32_t d;
    asm("v_pk_sub_i16 %0, %1, %2\n\tv_pk_ashrrev_i16 %0, 15, %0 op_sel_hi:[0,1]" : "=&v"(d) : "v"(a), "v"(b));
    return d;
}

// inclusive max scan over the 64 lanes (identity INT_MIN), DPP row_shr + row_bcast
__device__ __forceinline__ int wave_scan_max(int x)
{
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x118, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x142, 0xa, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x143, 0xc, 0xf, false));
    return x;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x)
{
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
// lane L gets lane L - 1's x (lane 0 gets `first`)
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t x, uint32_t first)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)x, 0x138, 0xf, 0xf, false);   // wave_shr:1
}
// lane L gets lane L + 1's x (lane 63 gets `last`)
__device__ __forceinline__ uint32_t from_next_lane(uint32_t x, uint32_t last)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)last, (int)x, 0x130, 0xf, 0xf, false);    // wave_shl:1
}

}  // namespace

// A.1 first-row value of column j: eh[j].h (E = 0)
__device__ __forceinline__ int wv_init_h(int j, int h0, int qlen, int oe_ins, int e_ins)
{
    return j == 0 ? h0 : (j <= qlen ? max(h0 - oe_ins - (j - 1) * e_ins, 0) : 0);
}

template <int C>
__global__ __launch_bounds__(64) void wv_kernel(const KParams kp, const int32_t w, SeqPair *__restrict__ pairs,
                                                const int32_t *__restrict__ order, const int32_t n,
                                                const uint8_t *__restrict__ ref, const uint8_t *__restrict__ qer,
                                                int32_t *__restrict__ err)
{
    static_assert(C == 4 || C == 8 || C == 16, "columns per lane");
    constexpr int R = C / 2;                       // packed registers per plane
    constexpr int WIN = 64 * C;
    __shared__ uint32_t s_q[kWvQmax / 4];          // the pair's query codes (bytes)
    __shared__ uint2 s_prof[8];
    const int ln = threadIdx.x;
    if (ln < 8) s_prof[ln] = make_uint2(kp.prof[ln][0], kp.prof[ln][1]);
    const int oe_del = kp.o_del + kp.e_del, oe_ins = kp.o_ins + kp.e_ins;
    const uint32_t oed2 = pk2(oe_del), oei2 = pk2(oe_ins - kp.e_ins), ed2 = pk2(kp.e_del);

    for (int k = blockIdx.x; k < n; k += gridDim.x) {
        const int idx = __builtin_amdgcn_readfirstlane(order ? order[k] : k);
        SeqPair *sp = pairs + idx;
        const int idr = __builtin_amdgcn_readfirstlane(sp->idr), idq = __builtin_amdgcn_readfirstlane(sp->idq);
        const int tlen = __builtin_amdgcn_readfirstlane(sp->len1), qlen = __builtin_amdgcn_readfirstlane(sp->len2);
        const int h0 = __builtin_amdgcn_readfirstlane(sp->h0);
        // A.2 band cap (integer form of (int)((double)N / e + 1.))
        int wl = w;
        {
            const int ni = qlen * kp.maxsc + kp.end_bonus - kp.o_ins;
            const int nd = qlen * kp.maxsc + kp.end_bonus - kp.o_del;
            wl = min(wl, max((ni + kp.e_ins) / kp.e_ins, 1));
            wl = min(wl, max((nd + kp.e_del) / kp.e_del, 1));
        }
        if (qlen < 0 || tlen < 0 || h0 < 0 || qlen > kWvQmax || 2 * wl + C + 2 > WIN) {
            if (ln == 0) atomicOr(err, 1);
            continue;
        }
        // query codes -> LDS (words past qlen read as 0 in lane_cols)
        __syncthreads();
        for (int b = ln; b < (qlen + 3) / 4; b += 64) {
            uint32_t v = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int j = 4 * b + t;
                if (j < qlen) v |= (uint32_t)qer[idq + j] << (8 * t);
            }
            s_q[b] = v;
        }
        __syncthreads();
        // window [wb, wb + WIN): lane ln holds columns j0 .. j0 + C - 1
        int wb = 0;
        uint32_t hh[R], ee[R], qs[C / 4], jj[R], kem[R];
        auto lane_cols = [&]() {                     // per-lane column constants and query codes
            const int j0 = wb + C * ln;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                jj[r] = (uint32_t)(j0 + 2 * r) | ((uint32_t)(j0 + 2 * r + 1) << 16);
                // (j - 1) e_ins, the F offset: F~(j) = P(j) - (j - 1) e
                kem[r] = (uint32_t)((j0 + 2 * r - 1) * kp.e_ins & 0xffff) |
                         ((uint32_t)((j0 + 2 * r) * kp.e_ins) << 16);
            }
#pragma unroll
            for (int g = 0; g < C / 4; ++g) {
                const int wi = (j0 >> 2) + g;
                const uint32_t c = 4 * wi < qlen ? s_q[wi] : 0u;
                qs[g] = __builtin_amdgcn_perm(c, c, 0x03010200u);          // {c0, c2, c1, c3}
            }
        };
        lane_cols();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int j = C * ln + 2 * r;
            hh[r] = (uint32_t)wv_init_h(j, h0, qlen, oe_ins, kp.e_ins) |
                    ((uint32_t)wv_init_h(j + 1, h0, qlen, oe_ins, kp.e_ins) << 16);
            ee[r] = 0;
        }
        int best = h0, best_i = -1, best_j = -1, max_ie = -1, gsc = -1, moff = 0, endc = qlen;
        const uint8_t *tp = ref + idr;
        const int tsh = (int)((uintptr_t)tp & 3);
        const uint32_t *twp = (const uint32_t *)(tp - tsh);        // aligned words holding the target
        const int tlast = max((tsh + tlen - 1) >> 2, 0);
        uint32_t tw0 = tlen > 0 ? twp[0] : 0u, tw1 = tlen > 0 ? twp[min(1, tlast)] : 0u;
        for (int i = 0; i < tlen; ++i) {
            const int beg = max(0, i - wl);
            const int end = min(min(endc, i + wl + 1), qlen);
            // slide the window so that it starts at the lane holding beg
            const int nb = (beg / C) * C;
            while (wb < nb) {                        // one lane per step (beg grows by <= 1 a row)
                wb += C;
                const int jn = wb + WIN - C;             // first column entering on lane 63
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int j = jn + 2 * r;
                    const uint32_t hin = (uint32_t)wv_init_h(j, h0, qlen, oe_ins, kp.e_ins) |
                                         ((uint32_t)wv_init_h(j + 1, h0, qlen, oe_ins, kp.e_ins) << 16);
                    hh[r] = from_next_lane(hh[r], hin);
                    ee[r] = from_next_lane(ee[r], 0u);
                }
                lane_cols();
            }
            // target base (uniform; the next word is prefetched 4 rows ahead) and its profile
            const int tb = tsh + i;
            if ((tb & 3) == 0 && i > 0) {
                tw0 = tw1;
                tw1 = twp[min((tb >> 2) + 1, tlast)];
            }
            const int t = min((int)((tw0 >> (8 * (tb & 3))) & 0xffu), 7);
            const uint2 pr = s_prof[t];
            const int h1b = beg == 0 ? max(h0 - (kp.o_del + kp.e_del * (i + 1)), 0) : 0;
            const uint32_t begw = pk2(beg), endw = pk2(end), endp1w = pk2(end + 1);
            uint32_t hnew[R], enew[R], me[R], u[R];
            // scores + phase 1
#pragma unroll
            for (int g = 0; g < C / 4; ++g) {
                const uint32_t y = __builtin_amdgcn_perm(pr.y, pr.x, qs[g]);
                uint32_t sa, sb;
                asm("v_pk_lshlrev_b16 %0, 8, %2 op_sel_hi:[0,1]\n\t"
                    "v_pk_ashrrev_i16 %0, 8, %0 op_sel_hi:[0,1]\n\t"
                    "v_pk_ashrrev_i16 %1, 8, %2 op_sel_hi:[0,1]"
                    : "=&v"(sa), "=&v"(sb) : "v"(y));
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int r = 2 * g + h;
                    const uint32_t s = h ? sb : sa;
                    const uint32_t m = padd(pmin(s, hh[r]), hh[r]);       // M = hold + min(S, hold)
                    me[r] = pmax(m, ee[r]);
                    enew[r] = pmax(psub(ee[r], ed2), psub(m, oed2));      // E' (unclamped)
                    // U(k) = M(k) - oe_ins + k e_ins = M(k) - (oe_ins - e_ins) + (k - 1) e_ins
                    // for k >= beg, -inf left of beg
                    const uint32_t uk = padd(psub(m, oei2), kem[r]);
                    const uint32_t lm = plt(jj[r], begw);                 // k < beg
                    u[r] = (uk & ~lm) | (pk2(kWvNeg) & lm);
                }
            }
            // F prefix: lane-local inclusive prefix, exclusive scan over lanes, then per column
            uint32_t v[R];
            v[0] = ppre(u[0]);
#pragma unroll
            for (int r = 1; r < R; ++r) v[r] = pmax_bhi(ppre(u[r]), v[r - 1]);
            const int tot = (int)v[R - 1] >> 16;                          // lane max of U (sext)
            const int inc = wave_scan_max(tot);
            const int pin = (int)from_prev_lane((uint32_t)inc, (uint32_t)kWvNeg);   // exclusive
            const uint32_t pw = pk2(max(pin, kWvNeg));
            uint32_t hcur[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                // exclusive prefix of the two columns: {pre(2r-1), pre(2r)} within the lane
                const uint32_t prev_hi = r == 0 ? pk2(kWvNeg) : v[r - 1];
                const uint32_t ex = __builtin_amdgcn_alignbyte(r == 0 ? u[0] : v[r], prev_hi, 2);
                // r == 0: {NEG, U(0)}; else {v[r-1].hi, v[r].lo}
                const uint32_t ex0 = r == 0 ? ((u[0] << 16) | (pk2(kWvNeg) & 0xffffu)) : ex;
                const uint32_t p = pmax(pw, ex0);
                const uint32_t f = pmax(psub(p, kem[r]), 0u);             // F = max(P - (j-1)e, 0)
                hcur[r] = pmax(me[r], f);                                 // H(i, j)
            }
            // hold(j) <- H(i, j - 1): shift one column right (lane 0 gets the boundary h1b)
            const uint32_t lastprev = from_prev_lane(hcur[R - 1], pk2(h1b));
#pragma unroll
            for (int r = 0; r < R; ++r)
                hnew[r] = __builtin_amdgcn_alignbyte(hcur[r], r == 0 ? lastprev : hcur[r - 1], 2);
            // writes: slots <= end (H), slots < end (E), E(end) = 0; slots > end stale
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t le = plt(jj[r], endp1w);                  // j <= end
                const uint32_t lt = plt(jj[r], endw);                    // j < end
                hh[r] = (hnew[r] & le) | (hh[r] & ~le);
                ee[r] = (enew[r] & lt) | (ee[r] & ~le);
            }
            // row max (last column on ties) over [beg, end)
            uint32_t key = 0, hm[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t in = plt(jj[r], endw) & ~plt(jj[r], begw);
                hm[r] = hcur[r] & in;
                key = max(key, __builtin_amdgcn_perm(hm[r], jj[r], 0x05040100u));   // H.lo << 16 | j
                key = max(key, __builtin_amdgcn_perm(hm[r], jj[r], 0x07060302u));   // H.hi << 16 | j+1
            }
            const uint32_t kmax = wave_max_u32(key);
            const int m = (int)(kmax >> 16), mj = (int)(kmax & 0xffffu);
            // h1 at row end = H(i, end - 1) (an empty row leaves h1 = h1b): one v_readlane
            int hq = h1b;
            if (end - 1 >= beg) {
                const int rel = end - 1 - wb, lane = rel / C, col = rel % C;
                uint32_t hv = 0;
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (col >> 1 == r) hv = hcur[r];
                const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)hv, lane);
                hq = (int)(int16_t)((col & 1) ? (x >> 16) : (x & 0xffffu));
            }
            if (end == qlen) {                       // A.4: j == qlen; h1 = H(i, qlen - 1)
                if (!(gsc > hq)) max_ie = i;
                gsc = max(gsc, hq);
            }
            if (m <= 0) break;
            if (m > best) {
                best = m; best_i = i; best_j = mj;
                moff = max(moff, abs(mj - i));
            } else if (kp.zdrop > 0) {
                const int di = i - best_i, dj = mj - best_j;
                const int dz = (di > dj) ? best - m - (di - dj) * kp.e_del : best - m - (dj - di) * kp.e_ins;
                if (dz > kp.zdrop) break;
            }
            // 1 + lastH: H(i, end - 1) > 0 gives lastH = end - 1 at once;
            // only rows whose band end shrinks pay the wave reduction of the last positive column
            int lp1 = end;
            if (hq <= 0) {
                uint32_t lp = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t plo = (hm[r] & 0xffffu) ? (jj[r] & 0xffffu) + 1u : 0u;
                    const uint32_t phi = (hm[r] >> 16) ? (jj[r] >> 16) + 1u : 0u;
                    lp = max(lp, max(plo, phi));
                }
                lp1 = (int)wave_max_u32(lp);
            }
            endc = min(lp1 + 2, qlen);
        }
        if (ln == 0) {
            sp->score = best;
            sp->tle = best_i + 1;
            sp->gtle = max_ie + 1;
            sp->qle = best_j + 1;
            sp->gscore = gsc;
            sp->max_off = moff;
        }
    }
}

hipError_t launch_wv_kernel(int cols, const KParams &kp, int32_t w, SeqPair *pairs, const int32_t *order,
                            int32_t n, const uint8_t *ref, const uint8_t *qer, int32_t *err, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    // one wave per pair, grid-stride over the class (enough waves to fill 256 CUs x 4 SIMDs x 8)
    const unsigned grid = (unsigned)min(n, 8192);
    switch (cols) {
    case 4: hipLaunchKernelGGL(wv_kernel<4>, dim3(grid), dim3(64), 0, s, kp, w, pairs, order, n, ref, qer, err); break;
    case 8: hipLaunchKernelGGL(wv_kernel<8>, dim3(grid), dim3(64), 0, s, kp, w, pairs, order, n, ref, qer, err); break;
    case 16: hipLaunchKernelGGL(wv_kernel<16>, dim3(grid), dim3(64), 0, s, kp, w, pairs, order, n, ref, qer, err); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace bsw
