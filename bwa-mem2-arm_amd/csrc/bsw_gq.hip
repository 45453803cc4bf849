// bsw_gq.hip -- the small-batch band kernel: one 16-lane ROW GROUP per SeqPair, four pairs per
// wavefront (gfx950).
//
// Why: upstream's kt_for workers hand getScores16/8 a few thousand pairs per call.  The lane
// kernels (bsw_pc.hip) keep a pair's whole row in ONE lane, so a wave lives as long as its
// pairs' rows x columns (~1.2 ms at C2) whatever the batch size; the wave-per-alignment kernel
// (bsw_wv.hip) spreads a pair over 64 lanes as a 64*C-column sliding window, most of it idle
// for a 150-column query, and pays two full-wave reductions per row.  Here a pair's whole query
// (<= 16*C columns, C <= 10: 160) sits in the 16 lanes of one DPP row, C columns per lane, so:
//   - no window slides (the band never leaves the resident row);
//   - every cross-lane step is a DPP op inside the 16-lane row: the F prefix is a 4-step
//     row_shr scan, the H shift one row_shr:1, the row-max key a 4-step row_ror all-reduce --
//     no row_bcast, no v_readlane, no scalar chain between rows;
//   - the per-pair bookkeeping (band, best, z-drop, gscore, max_off) runs as VALU in the group's
//     lanes, so the four pairs of a wave are independent: a pair that breaks is masked off.
// Cell arithmetic is bsw_wv.hip's (ksw_extend2 exact): two columns per v_pk_* op,
//     M = hold + min(S, hold)  (max(mat) == 1),  E' = max(E - e_del, M - oe_del) (unclamped),
//     F(j) = max(0, P(j) - (j-1) e_ins), P(j) = max_{beg <= k < j} (M(k) - oe_ins + k e_ins),
//     H = max(M, E, F);  writes only to slots <= end (A.7 stale columns), E(end) = 0;
//     row max with the LAST column on ties by the key H << 16 | j.
// Contract (gq_eligible): max(mat) == 1, qlen <= 16*C, the wave kernel's int16 bounds.  Pairs
// that do not qualify are skipped and raise *flag (the host then runs the batch on the planned
// path); with flag == nullptr they raise the range guard *err instead.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "bsw_kernels.h"

namespace bsw {

namespace {

constexpr int kGqNeg = -30000;                 // "-inf" of the F prefix (int16 lanes)

__device__ __forceinline__ uint32_t pk2(int v) { return ((uint32_t)v & 0xffffu) * 0x10001u; }

#define GQ_OP2(name, ins)                                                                    \
    __device__ __forceinline__ uint32_t name(uint32_t a, uint32_t b)                        \
    {                                                                                        \
        uint32_t d;                                                                          \
        asm(ins " %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));                                   \
        return d;                                                                            \
    }
GQ_OP2(pmax, "v_pk_max_i16")
GQ_OP2(pmin, "v_pk_min_i16")
GQ_OP2(padd, "v_pk_add_u16")
GQ_OP2(psub, "v_pk_sub_i16")
GQ_OP2(pmaxu, "v_pk_max_u16")
#undef GQ_OP2

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
// (m & a) | (~m & b)
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }

// DPP inside each group.  GS = 16: the group is one DPP row (row_shr / row_ror); values are kept
// non-negative where a scan needs an identity, so out-of-row sources read as 0 (bound_ctrl) and
// every step folds into one v_max_*_dpp.  GS = 4: the group is a quad (quad_perm; a max scan may
// let lane 0 read itself, max being idempotent).
#define GQ_SHR0(x, n) __builtin_amdgcn_update_dpp(0, (x), 0x110 + (n), 0xf, 0xf, true)
#define GQ_ROR(x, n) __builtin_amdgcn_update_dpp(0, (x), 0x120 + (n), 0xf, 0xf, false)
#define GQ_QP(x, ctl) __builtin_amdgcn_update_dpp(0, (x), (ctl), 0xf, 0xf, false)
constexpr int kQpShr1 = 0x90;                      // quad_perm [0, 0, 1, 2]
constexpr int kQpShr2 = 0x40;                      // quad_perm [0, 0, 0, 1]
constexpr int kQpXor1 = 0xB1;                      // quad_perm [1, 0, 3, 2]
constexpr int kQpXor2 = 0x4E;                      // quad_perm [2, 3, 0, 1]

// GS = 32: two DPP rows per group -- the scans end with row_bcast:15 (row 2k's last lane into
// row 2k + 1), the one-lane shift is wave_shr:1 (then lane 0 of each group cleared), the all-reduce
// ends with v_permlane16_swap (rows 2k <-> 2k + 1)
#define GQ_BC15(x) __builtin_amdgcn_update_dpp(0, (x), 0x142, 0xa, 0xf, false)
#define GQ_WSHR1(x) __builtin_amdgcn_update_dpp(0, (x), 0x138, 0xf, 0xf, true)

// inclusive max scan over the group's lanes of non-negative x
template <int GS>
__device__ __forceinline__ int grp_scan_max0(int x)
{
    if constexpr (GS == 16 || GS == 32) {
        x = max(x, GQ_SHR0(x, 1));
        x = max(x, GQ_SHR0(x, 2));
        x = max(x, GQ_SHR0(x, 4));
        x = max(x, GQ_SHR0(x, 8));
        if constexpr (GS == 32) x = max(x, GQ_BC15(x));
    } else {
        x = max(x, GQ_QP(x, kQpShr1));
        x = max(x, GQ_QP(x, kQpShr2));
    }
    return x;
}
// lane l gets lane l - 1's x inside the group; lane 0 gets 0
template <int GS>
__device__ __forceinline__ int grp_shr1_0(int x, int gl)
{
    if constexpr (GS == 16) return GQ_SHR0(x, 1);
    else if constexpr (GS == 32) {
        const int y = GQ_WSHR1(x);
        return gl == 0 ? 0 : y;
    } else {
        const int y = GQ_QP(x, kQpShr1);
        return gl == 0 ? 0 : y;
    }
}
// unsigned max over the group's lanes, result in every lane of the group
template <int GS>
__device__ __forceinline__ uint32_t grp_max_u32(uint32_t x)
{
    if constexpr (GS == 16 || GS == 32) {
        x = max(x, (uint32_t)GQ_ROR((int)x, 8));
        x = max(x, (uint32_t)GQ_ROR((int)x, 4));
        x = max(x, (uint32_t)GQ_ROR((int)x, 2));
        x = max(x, (uint32_t)GQ_ROR((int)x, 1));
        if constexpr (GS == 32) {
            const auto sw = __builtin_amdgcn_permlane16_swap(x, x, false, false);
            x = max((uint32_t)sw[0], (uint32_t)sw[1]);
        }
    } else {
        x = max(x, (uint32_t)GQ_QP((int)x, kQpXor1));
        x = max(x, (uint32_t)GQ_QP((int)x, kQpXor2));
    }
    return x;
}

__device__ __forceinline__ int gq_init_h(int j, int h0, int qlen, int oe_ins, int e_ins)
{
    return j == 0 ? h0 : (j <= qlen ? max(h0 - oe_ins - (j - 1) * e_ins, 0) : 0);
}

}  // namespace

// Targets are staged in LDS (a global-load prefetch would be waited for at the loop's register
// copy in the same row), so a target longer than gq_tmax(GS) takes the planned path: 1 KB per
// pair for 16-lane groups (4 per wave), 512 B for quads (16 per wave: 8 KB of LDS per wave).
__host__ __device__ constexpr int gq_tmax(int gs) { return gs >= 16 ? 1024 : 512; }

// Same int16 bounds as the wave kernel (bsw_host.cpp wv_class); the whole query is resident,
// so the band cap only limits [beg, end).
__host__ __device__ __forceinline__ bool gq_eligible(const KParams &kp, int qlen, int tlen, int h0, int qmax,
                                                     int tmax)
{
    if (kp.maxsc != 1 || qlen < 0 || tlen < 0 || h0 < 0 || qlen > qmax || tlen > tmax) return false;
    if ((int64_t)kp.e_ins * qlen >= 2700) return false;
    if (128 + kp.o_del + 2 * kp.e_del >= 30000 || 128 + kp.o_ins + 2 * kp.e_ins >= 30000) return false;
    if ((int64_t)h0 + (qlen < tlen ? qlen : tlen) + (int64_t)kp.e_ins * (qlen + 1) >= 30000) return false;
    return true;
}

template <int C, int GS>
__global__ __launch_bounds__(64) void gq_kernel(const KParams kp, const int32_t w, SeqPair *__restrict__ pairs,
                                                const int32_t *__restrict__ order, const int32_t n,
                                                const uint8_t *__restrict__ ref, const uint8_t *__restrict__ qer,
                                                int32_t *__restrict__ err, int32_t *__restrict__ flag,
                                                int32_t *__restrict__ out24)
{
    static_assert((GS == 16 && (C == 4 || C == 6 || C == 8 || C == 10)) ||
                  (GS == 32 && (C == 2 || C == 4 || C == 6)) ||
                  (GS == 4 && (C == 16 || C == 24 || C == 32 || C == 40)), "group size / columns per lane");
    constexpr int R = C / 2;                       // packed registers per plane
    constexpr int G = (C + 3) / 4;                 // query words per lane (4 codes each)
    constexpr int QMAX = GS * C;
    constexpr int NG = 64 / GS;                    // pairs per wave
    constexpr int TW = gq_tmax(GS) / 4 + 2;        // target words per group (+ alignment slack)
    __shared__ uint2 s_prof[8];
    __shared__ uint32_t s_t[NG][TW];               // the wave's pairs' targets (aligned words)
    if (threadIdx.x < 8) s_prof[threadIdx.x] = make_uint2(kp.prof[threadIdx.x][0], kp.prof[threadIdx.x][1]);
    const int gl = threadIdx.x & (GS - 1);         // lane in the group
    const int grp = threadIdx.x / GS;
    const int k = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / GS);   // pair slot
    const int oe_del = kp.o_del + kp.e_del, oe_ins = kp.o_ins + kp.e_ins;
    const uint32_t oed2 = pk2(oe_del), oei2 = pk2(oe_ins - kp.e_ins), ed2 = pk2(kp.e_del);
    // the z-drop's gap extensions as values pinned in registers: with the plain `c ? x * kp.e_del :
    // y * kp.e_ins` the compiler selected between the two fields' ADDRESSES and issued a vector load
    // from the kernarg segment every row, waited for at once (vmcnt(0): an L2 round trip per row)
    int zd_del = kp.e_del, zd_ins = kp.e_ins;
    asm volatile("" : "+s"(zd_del), "+s"(zd_ins));

    int idx = -1, idr = 0, idq = 0, tlen = 0, qlen = 0, h0 = 0;
    bool alive = false;
    if (k < n) {
        idx = order ? order[k] : k;
        const SeqPair &sp = pairs[idx];
        idr = sp.idr; idq = sp.idq; tlen = sp.len1; qlen = sp.len2; h0 = sp.h0;
        alive = gq_eligible(kp, qlen, tlen, h0, QMAX, gq_tmax(GS));
        if (!alive && gl == 0) atomicOr(flag ? flag : err, 1);
        if (!alive) idx = -1;
    }
    // the target's aligned words -> LDS (the group's lanes); byte tsh + i is row i's base
    const uint8_t *tp = ref + (alive ? idr : 0);
    const int tsh = (int)((uintptr_t)tp & 3);
    if (alive) {
        const uint32_t *twp = (const uint32_t *)(tp - tsh);
        const int nw = (tsh + tlen + 3) >> 2;
        for (int b = gl; b < nw; b += GS) s_t[grp][b] = twp[b];
    }
    __syncthreads();
    const uint8_t *tb8 = (const uint8_t *)s_t[grp] + tsh;
    // A.2 band cap (integer form of (int)((double)N / e + 1.))
    int wl = w;
    {
        const int ni = qlen * kp.maxsc + kp.end_bonus - kp.o_ins;
        const int nd = qlen * kp.maxsc + kp.end_bonus - kp.o_del;
        wl = min(wl, max((ni + kp.e_ins) / kp.e_ins, 1));
        wl = min(wl, max((nd + kp.e_del) / kp.e_del, 1));
    }
    const int j0 = C * gl;
    uint32_t hh[R], ee[R], qs[G], jj[R], kem[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = j0 + 2 * r;
        jj[r] = (uint32_t)j | ((uint32_t)(j + 1) << 16);
        kem[r] = (uint32_t)((j - 1) * kp.e_ins & 0xffff) | ((uint32_t)(j * kp.e_ins) << 16);
        hh[r] = alive ? ((uint32_t)gq_init_h(j, h0, qlen, oe_ins, kp.e_ins) & 0xffffu) |
                            ((uint32_t)gq_init_h(j + 1, h0, qlen, oe_ins, kp.e_ins) << 16)
                      : 0u;
        ee[r] = 0;
    }
    // the lane's query codes (columns past qlen read as 0: never inside [beg, end))
#pragma unroll
    for (int g = 0; g < G; ++g) {
        uint32_t c = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = j0 + 4 * g + t;
            if (alive && j < qlen) c |= (uint32_t)qer[idq + j] << (8 * t);
        }
        qs[g] = __builtin_amdgcn_perm(c, c, 0x03010200u);          // {c0, c2, c1, c3}
    }
    // row i's profile, read from LDS one row ahead
    uint2 pr = s_prof[alive && tlen > 0 ? min((int)tb8[0], 7) : 0];

    // static per lane: columns inside the query, and where column qlen - 1 lives (the row end
    // of every row whose band reaches qlen)
    uint32_t colm[R];
#pragma unroll
    for (int r = 0; r < R; ++r) colm[r] = plt(jj[r], pk2(qlen));             // j < qlen
    const int qc = qlen - 1;
    const int qr = (qc >= 0 && qc / C == gl) ? (qc % C) >> 1 : -1;          // register holding it
    const int qsh = (qc & 1) * 16;

    int best = h0, best_i = -1, best_j = -1, max_ie = -1, gsc = -1, moff = 0, endc = qlen;
    int i = 0;
    // One row.  LM: some live pair has beg > 0 (columns left of beg are masked out of the F chain
    // and the key).  RM: some live pair's band ends before qlen, so writes stop at slot end and E(end)
    // = 0 (A.7 stale columns); without it every pair's end is qlen and slots past qlen are never
    // read, so the row writes unmasked and finds H(i, qlen - 1) at a fixed place.
    // K8 (every pair of the wave has H <= h0 + min(qlen, tlen) <= 255): the row-max key as two
    // 16-bit halves H << 8 | j per register (one v_perm + one v_pk_max_u16) instead of two 32-bit
    // keys H << 16 | j (two v_perm + two v_max); folded to one 32-bit key before the group
    // reduction, same last-column tie rule
    auto row = [&](auto LMc, auto RMc, auto K8c) {
        constexpr bool LM = decltype(LMc)::value, RM = decltype(RMc)::value, K8 = decltype(K8c)::value;
        const uint2 prn = s_prof[min((int)tb8[min(i + 1, tlen - 1)], 7)];
        const int beg = max(0, i - wl);
        const int end = min(min(endc, i + wl + 1), qlen);
        const int h1b = beg == 0 ? max(h0 - (kp.o_del + kp.e_del * (i + 1)), 0) : 0;
        const uint32_t begw = pk2(beg), endw = pk2(end), endp1w = pk2(end + 1);
        uint32_t enew[R], me[R], u[R], lm[R];
        // scores + phase 1
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t y = __builtin_amdgcn_perm(pr.y, pr.x, qs[g]);
            uint32_t sa, sb;
            asm("v_pk_lshlrev_b16 %0, 8, %2 op_sel_hi:[0,1]\n\t"
                "v_pk_ashrrev_i16 %0, 8, %0 op_sel_hi:[0,1]\n\t"
                "v_pk_ashrrev_i16 %1, 8, %2 op_sel_hi:[0,1]"
                : "=&v"(sa), "=&v"(sb) : "v"(y));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int r = 2 * g + h;
                if (r >= R) break;
                const uint32_t sc = h ? sb : sa;
                const uint32_t m = padd(pmin(sc, hh[r]), hh[r]);      // M = hold + min(S, hold)
                me[r] = pmax(m, ee[r]);
                enew[r] = pmax(psub(ee[r], ed2), psub(m, oed2));      // E' (unclamped)
                const uint32_t uk = padd(psub(m, oei2), kem[r]);      // U(k) = M(k) - oe + k e
                if constexpr (LM) {
                    lm[r] = plt(jj[r], begw);                         // k < beg
                    u[r] = bsel(lm[r], pk2(kGqNeg), uk);
                } else {
                    lm[r] = 0;
                    u[r] = uk;
                }
            }
        }
        pr = prn;
        // F prefix: lane-local inclusive prefix, exclusive scan over the group's lanes (on
        // U - kGqNeg >= 0, so out-of-row DPP sources read as the identity 0)
        uint32_t v[R];
        v[0] = ppre(u[0]);
#pragma unroll
        for (int r = 1; r < R; ++r) v[r] = pmax_bhi(ppre(u[r]), v[r - 1]);
        const int tot = ((int)v[R - 1] >> 16) - kGqNeg;               // lane max of U, offset
        const int inc = grp_scan_max0<GS>(tot);
        const int pin = grp_shr1_0<GS>(inc, gl) + kGqNeg;             // exclusive (lane 0: NEG)
        const uint32_t pw = pk2(pin);
        uint32_t hcur[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t ex0 = r == 0 ? ((u[0] << 16) | (pk2(kGqNeg) & 0xffffu))
                                        : __builtin_amdgcn_alignbyte(v[r], v[r - 1], 2);   // {v[r-1].hi, v[r].lo}
            const uint32_t p = pmax(pw, ex0);
            const uint32_t f = pmax(psub(p, kem[r]), 0u);             // F = max(P - (j-1)e, 0)
            hcur[r] = pmax(me[r], f);                                 // H(i, j)
        }
        // hold(j) <- H(i, j - 1): one column right (group lane 0 gets the boundary h1b)
        const uint32_t shf = (uint32_t)grp_shr1_0<GS>((int)hcur[R - 1], gl);
        const uint32_t lastprev = gl == 0 ? pk2(h1b) : shf;
        // writes: slots <= end (H), slots < end (E), E(end) = 0; slots > end stale.  Row max
        // key (last column on ties) over [beg, end); H(i, end - 1) for gscore / lastH
        uint32_t key = 0, hq_c = 0, hsel = 0, lt[R];
        const int rel = end - 1 - j0;                                 // column end-1 in this lane?
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t hn = __builtin_amdgcn_alignbyte(hcur[r], r == 0 ? lastprev : hcur[r - 1], 2);
            if constexpr (RM) {
                const uint32_t le = plt(jj[r], endp1w);              // j <= end
                lt[r] = plt(jj[r], endw);                            // j < end
                hh[r] = bsel(le, hn, hh[r]);
                ee[r] = bsel(le, enew[r] & lt[r], ee[r]);
                hq_c = rel == 2 * r ? (hcur[r] & 0xffffu) : hq_c;
                hq_c = rel == 2 * r + 1 ? (hcur[r] >> 16) : hq_c;
            } else {
                lt[r] = colm[r];                                     // end == qlen
                hh[r] = hn;
                ee[r] = enew[r];
                hsel = qr == r ? hcur[r] : hsel;
            }
            const uint32_t hm = LM ? (hcur[r] & lt[r] & ~lm[r]) : (hcur[r] & lt[r]);
            if constexpr (K8)
                key = pmaxu(key, __builtin_amdgcn_perm(hm, jj[r], 0x06020400u));    // {H << 8 | j} x 2
            else
                key = max(key, max(__builtin_amdgcn_perm(hm, jj[r], 0x05040100u),     // H.lo << 16 | j
                                   __builtin_amdgcn_perm(hm, jj[r], 0x07060302u)));   // H.hi << 16 | j+1
        }
        if constexpr (!RM) hq_c = qr >= 0 ? (hsel >> qsh) & 0xffffu : 0u;
        if constexpr (K8) key = max(key & 0xffffu, key >> 16);
        const uint32_t kmax = grp_max_u32<GS>(key);
        const int m = (int)(kmax >> (K8 ? 8 : 16)), mj = (int)(kmax & (K8 ? 0xffu : 0xffffu));
        int hq = (int)grp_max_u32<GS>(hq_c);                              // H >= 0 in [beg, end)
        hq = end - 1 < beg ? h1b : hq;                                // empty row: h1 = h1b
        // A.4: j == qlen (gscore, max_ie) -- selects, no exec-masked blocks
        const bool atq = end == qlen;
        max_ie = (atq && !(gsc > hq)) ? i : max_ie;
        gsc = atq ? max(gsc, hq) : gsc;
        const bool better = m > best;                                 // implies m > 0 (best >= 0)
        const int di = i - best_i, dj = mj - best_j;
        const int dz = best - m - ((di > dj) ? (di - dj) * zd_del : (dj - di) * zd_ins);
        const bool stop = m <= 0 || (!better && kp.zdrop > 0 && dz > kp.zdrop);
        moff = better ? max(moff, abs(mj - i)) : moff;
        best_i = better ? i : best_i;
        best_j = better ? mj : best_j;
        best = better ? m : best;
        // 1 + lastH: H(i, end - 1) > 0 gives lastH = end - 1; groups
        // whose band end shrinks reduce the last positive column of the row
        int lp1 = end;
        const bool shrink = hq <= 0;
        if (__builtin_amdgcn_ballot_w64(shrink && !stop)) {
            uint32_t lp = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t hm = LM ? (hcur[r] & lt[r] & ~lm[r]) : (hcur[r] & lt[r]);
                const uint32_t plo = (hm & 0xffffu) ? (jj[r] & 0xffffu) + 1u : 0u;
                const uint32_t phi = (hm >> 16) ? (jj[r] >> 16) + 1u : 0u;
                lp = max(lp, max(plo, phi));
            }
            lp = grp_max_u32<GS>(lp);
            lp1 = shrink ? (int)lp : lp1;
        }
        endc = min(lp1 + 2, qlen);
        alive = alive && !stop;
    };
    const bool k8 = __builtin_amdgcn_ballot_w64(alive && h0 + min(qlen, tlen) > 255) == 0;
    auto rows = [&](auto K8c) {
        for (;; ++i) {
            const bool live = alive && i < tlen;
            if (!__builtin_amdgcn_ballot_w64(live)) break;
            // wave-uniform row forms (the masks only where some live pair needs them)
            const bool need_lm = __builtin_amdgcn_ballot_w64(live && i - wl > 0) != 0;
            const bool need_rm = __builtin_amdgcn_ballot_w64(live && min(min(endc, i + wl + 1), qlen) != qlen) != 0;
            if (!live) continue;
            if (need_rm) row(std::true_type{}, std::true_type{}, K8c);
            else if (need_lm) row(std::true_type{}, std::false_type{}, K8c);
            else row(std::false_type{}, std::false_type{}, K8c);
        }
    };
    if constexpr (GS >= 16) {         // (the quad form keeps one path: its registers are the limit)
        if (k8) rows(std::true_type{});
        else rows(std::false_type{});
    } else {
        (void)k8;
        rows(std::false_type{});
    }
    if (idx >= 0 && gl == 0) {
        if (out24) {
            int32_t *o = out24 + 6 * (int64_t)idx;
            o[0] = best; o[1] = best_i + 1; o[2] = max_ie + 1; o[3] = best_j + 1; o[4] = gsc; o[5] = moff;
        } else {
            SeqPair *sp = pairs + idx;
            sp->score = best;
            sp->tle = best_i + 1;
            sp->gtle = max_ie + 1;
            sp->qle = best_j + 1;
            sp->gscore = gsc;
            sp->max_off = moff;
        }
    }
}

int gq_cols_for(int max_qlen, int gs)
{
    if (gs == 32) {                      // latency form: two DPP rows per pair, 2 pairs per wave
        if (max_qlen <= 64) return 2;
        if (max_qlen <= 128) return 4;
        if (max_qlen <= 160) return 6;
        return -1;
    }
    if (gs == 16) {
        if (max_qlen <= 64) return 4;
        if (max_qlen <= 96) return 6;
        if (max_qlen <= 128) return 8;
        if (max_qlen <= 160) return 10;
    } else {
        if (max_qlen <= 64) return 16;
        if (max_qlen <= 96) return 24;
        if (max_qlen <= 128) return 32;
        if (max_qlen <= 160) return 40;
    }
    return -1;
}

bool gq_pair_ok(const KParams &kp, int qlen, int tlen, int h0, int gs)
{
    return gq_eligible(kp, qlen, tlen, h0, 160, gq_tmax(gs));
}

hipError_t launch_gq_kernel(int gs, int cols, const KParams &kp, int32_t w, SeqPair *pairs, const int32_t *order,
                            int32_t n, const uint8_t *ref, const uint8_t *qer, int32_t *err, int32_t *flag,
                            int32_t *out24, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    // one wave per workgroup: 64 / gs pairs (a small batch spreads over every CU)
    const int per = 64 / gs;
    const unsigned grid = (unsigned)((n + per - 1) / per);
#define GQ_L(C, GS) hipLaunchKernelGGL((gq_kernel<C, GS>), dim3(grid), dim3(64), 0, s, kp, w, pairs, order, n, ref, qer, \
                                       err, flag, out24)
    switch (gs * 100 + cols) {
    case 1604: GQ_L(4, 16); break;
    case 1606: GQ_L(6, 16); break;
    case 1608: GQ_L(8, 16); break;
    case 1610: GQ_L(10, 16); break;
    case 3202: GQ_L(2, 32); break;
    case 3204: GQ_L(4, 32); break;
    case 3206: GQ_L(6, 32); break;
    case 416: GQ_L(16, 4); break;
    case 424: GQ_L(24, 4); break;
    case 432: GQ_L(32, 4); break;
    case 440: GQ_L(40, 4); break;
    default: return hipErrorInvalidValue;
    }
#undef GQ_L
    return hipGetLastError();
}

}  // namespace bsw
