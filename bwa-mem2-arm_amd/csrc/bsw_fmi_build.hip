// bsw_fmi_build.hip -- FM-index construction on the GPU (bsw_fmi_internal.h fmi_build_gpu;
// DESIGN.md §4.12).  What makes a GRCh38-sized (3 Gb, two strands: 6 G suffixes) index
// buildable in seconds and resident in one MI355X's HBM (64-bit suffix array 48 GB + 6 GB of
// occurrence blocks + 6 GB of BWT codes, of 288 GB):
//   1. T = ref + revcomp(ref) written in HBM (the reference goes up once).
//   2. Suffixes bucketed by their first 3 bases (base-5 digits, '$' / past-the-end = 0: 125
//      buckets in lexicographic order): one histogram pass (LDS bins, one global atomic per bin
//      and block) and one scatter pass (block-local cursors) -- every bucket holds < 2^31
//      suffixes, which is what hipCUB's radix sort takes.
//   3. Per bucket: the 27-base key of every suffix (5^27 < 2^63), a 63-bit radix sort of
//      (key, position) pairs, positions written back in order.  Suffixes that reach '$' inside
//      their key are already totally ordered by it.
//   4. Tie groups (equal 27-base keys: chance repeats, copies): sorted by comparing the
//      suffixes themselves from base 27 on -- one thread per group of <= 32, the host's
//      std::sort for larger ones (long homopolymers / tandem repeats).
//   5. BWT codes (4 = '$'), the sentinel row, and 64-row occurrence blocks: per block the four
//      one-hot masks and counts, then one exclusive scan per code for the running counts.
// The suffix array equals the host prefix-doubling builder's (tests/test_fmi.py checks it).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <algorithm>
#include <type_traits>
#include <vector>
#include "bsw_fmi_internal.h"

namespace {

constexpr int kBuckets = 125;                      // 5^3

// A dispatch holds at most 2^32 - 1 work-items (the AQL packet's 32-bit grid size), and a 3 Gb
// genome has 6 G rows: every kernel over rows / text positions is grid-stride (kStrideGrid
// blocks of 256).
constexpr unsigned kStrideGrid = 1u << 20;

__global__ void k_make_text(const uint8_t *__restrict__ ref, int64_t len, uint8_t *__restrict__ T)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t c = ref[i];
        T[i] = c;
        T[2 * len - 1 - i] = (uint8_t)(3 - c);
    }
}

__device__ __forceinline__ uint64_t key27(const uint8_t *__restrict__ T, int64_t n, int64_t p)
{
    uint64_t k = 0;
#pragma unroll
    for (int d = 0; d < 27; ++d) {
        const int64_t q = p + d;
        k = k * 5 + (q < n ? (uint64_t)T[q] + 1 : 0);
    }
    return k;
}

__device__ __forceinline__ int bucket_of(const uint8_t *__restrict__ T, int64_t n, int64_t p)
{
    int b = 0;
#pragma unroll
    for (int d = 0; d < 3; ++d) b = b * 5 + (p + d < n ? T[p + d] + 1 : 0);
    return b;
}

__global__ void k_hist(const uint8_t *__restrict__ T, int64_t n, unsigned long long *__restrict__ cnt)
{
    __shared__ unsigned int s[kBuckets];
    for (int k = threadIdx.x; k < kBuckets; k += blockDim.x) s[k] = 0;
    __syncthreads();
    const int64_t N = n + 1;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&s[bucket_of(T, n, p)], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < kBuckets; k += blockDim.x)
        if (s[k]) atomicAdd(&cnt[k], (unsigned long long)s[k]);
}

// each block scatters a contiguous range of positions into the buckets (block-local cursors)
template <class S>
__global__ void k_scatter(const uint8_t *__restrict__ T, int64_t n, int64_t per_block,
                          unsigned long long *__restrict__ cursor, S *__restrict__ sa)
{
    __shared__ unsigned int cnt[kBuckets];
    __shared__ unsigned long long base[kBuckets];
    for (int k = threadIdx.x; k < kBuckets; k += blockDim.x) cnt[k] = 0;
    __syncthreads();
    const int64_t N = n + 1, p0 = (int64_t)blockIdx.x * per_block, p1 = min(N, p0 + per_block);
    for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) atomicAdd(&cnt[bucket_of(T, n, p)], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < kBuckets; k += blockDim.x) {
        base[k] = cnt[k] ? atomicAdd(&cursor[k], (unsigned long long)cnt[k]) : 0ull;
        cnt[k] = 0;
    }
    __syncthreads();
    for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        const int b = bucket_of(T, n, p);
        sa[base[b] + atomicAdd(&cnt[b], 1u)] = (S)p;
    }
}

template <class S>
__global__ void k_keys(const uint8_t *__restrict__ T, int64_t n, const S *__restrict__ pos, int64_t m,
                       uint64_t *__restrict__ key)
{
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) key[j] = key27(T, n, (int64_t)pos[j]);
}

// tie groups of a sorted bucket: [j0, j1) with equal keys, listed by their first index
__global__ void k_ties(const uint64_t *__restrict__ key, int64_t m, int64_t *__restrict__ grp, int64_t cap,
                       unsigned long long *__restrict__ ng)
{
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j + 1 >= m) return;
    if (key[j] == key[j + 1] && (j == 0 || key[j - 1] != key[j])) {
        int64_t e = j + 2;
        while (e < m && key[e] == key[j]) ++e;
        const unsigned long long g = atomicAdd(ng, 1ull);
        if ((int64_t)g < cap) {
            grp[2 * g] = j;
            grp[2 * g + 1] = e;
        }
    }
}

// suffix a < suffix b on T$, both known equal on their first `from` bases
__device__ __host__ __forceinline__ bool suffix_less(const uint8_t *T, int64_t n, int64_t a, int64_t b, int from)
{
    a += from;
    b += from;
    while (a < n && b < n) {
        if (T[a] != T[b]) return T[a] < T[b];
        ++a;
        ++b;
    }
    return a == n && b != n;         // the shorter remainder reaches '$' first
}

template <class S>
__global__ void k_sort_small_groups(const uint8_t *__restrict__ T, int64_t n, S *__restrict__ pos,
                                    const int64_t *__restrict__ grp, int64_t ng)
{
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ng) return;
    const int64_t a = grp[2 * g], b = grp[2 * g + 1];
    if (b - a > 32) return;                            // the host takes large groups
    for (int64_t i = a + 1; i < b; ++i) {
        const S v = pos[i];
        int64_t j = i - 1;
        while (j >= a && suffix_less(T, n, (int64_t)v, (int64_t)pos[j], 27)) {
            pos[j + 1] = pos[j];
            --j;
        }
        pos[j + 1] = v;
    }
}

template <class S>
__global__ void k_bwt(const uint8_t *__restrict__ T, const S *__restrict__ sa, int64_t N, uint8_t *__restrict__ bwt,
                      unsigned long long *__restrict__ sentinel)
{
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = (int64_t)sa[r];
        bwt[r] = p == 0 ? 4 : T[p - 1];
        if (p == 0) *sentinel = (unsigned long long)r;
    }
}

// masks and per-block counts (cnt[c * nb + b]); one thread per block of 64 rows
template <class B>
__global__ void k_blocks(const uint8_t *__restrict__ bwt, int64_t N, int64_t nb, B *__restrict__ blk,
                         unsigned long long *__restrict__ cnt)
{
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    uint64_t m[4] = {0, 0, 0, 0};
    for (int y = 0; y < 64; ++y) {
        const int64_t r = b * 64 + y;
        if (r >= N) break;
        const uint8_t c = bwt[r];
        if (c < 4) m[c] |= 1ull << y;
    }
    for (int c = 0; c < 4; ++c) {
        blk[b].bits[c] = m[c];
        cnt[c * nb + b] = (unsigned long long)__builtin_popcountll(m[c]);
    }
}

template <class B>
__global__ void k_block_counts(int64_t nb, const unsigned long long *__restrict__ pre, B *__restrict__ blk)
{
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    using C = std::remove_extent_t<decltype(B::cnt)>;
    for (int c = 0; c < 4; ++c) blk[b].cnt[c] = (C)pre[c * nb + b];
    if constexpr (sizeof(blk[b].cnt[0]) == 4) {
        for (int c = 0; c < 4; ++c) blk[b].pad[c] = 0;
    }
}

// ---- index self-check (bsw_fmi_check): every invariant the seeding walk relies on
// blocks: cnt[b + 1] = cnt[b] + popcount(bits[b]) per code, the last block's totals = count[]
template <class B>
__global__ void k_chk_blocks(const B *__restrict__ blk, int64_t nb, const int64_t *__restrict__ count,
                             unsigned long long *__restrict__ bad)
{
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    for (int c = 0; c < 4; ++c) {
        const uint64_t next = (uint64_t)blk[b].cnt[c] + (uint64_t)__builtin_popcountll(blk[b].bits[c]);
        const uint64_t want = b + 1 < nb ? (uint64_t)blk[b + 1].cnt[c] : (uint64_t)(count[c + 1] - count[c]);
        if (next != want) atomicAdd(bad, 1ull);
    }
}
// SA is a permutation of [0, n]; LF(r) = count[c] + Occ(c, r) with c = BWT[r] satisfies
// SA[LF(r)] = SA[r] - 1 for every row but the sentinel's (c = '$')
template <class S, class B>
__global__ void k_chk_lf(const S *__restrict__ sa, const uint8_t *__restrict__ bwt, const B *__restrict__ blk,
                         int64_t N, const int64_t *__restrict__ count, unsigned int *__restrict__ seen,
                         unsigned long long *__restrict__ bad)
{
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N; r += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t p = (uint64_t)sa[r];
        if (p >= (uint64_t)N) { atomicAdd(bad, 1ull); continue; }
        if (atomicOr(&seen[p >> 5], 1u << (p & 31)) & (1u << (p & 31))) atomicAdd(bad, 1ull);
        const int c = bwt[r];
        if (c > 4 || (c == 4) != (p == 0)) { atomicAdd(bad, 1ull); continue; }
        if (c == 4) continue;
        const B &k = blk[r >> 6];
        const uint64_t m = (r & 63) ? (~0ull >> (64 - (r & 63))) : 0ull;
        const int64_t lf = count[c] + (int64_t)k.cnt[c] + __builtin_popcountll(k.bits[c] & m);
        if (lf < 0 || lf >= N || (uint64_t)sa[lf] != p - 1) atomicAdd(bad, 1ull);
    }
}

int hrc(hipError_t e) { return e == hipSuccess ? BSW_OK : (e == hipErrorOutOfMemory ? BSW_E_NOMEM : BSW_E_HIP); }
#define FB_TRY(x)                             \
    do {                                      \
        const int rc_ = hrc(x);               \
        if (rc_) return rc_;                  \
    } while (0)

inline unsigned grid_of(int64_t n, int bs = 256) { return (unsigned)std::max<int64_t>(1, (n + bs - 1) / bs); }
inline unsigned stride_grid(int64_t n) { return std::min<unsigned>(grid_of(n), kStrideGrid); }

struct Scratch {                                       // temporaries of one build, freed on every path
    std::vector<void *> p;
    template <class T>
    hipError_t get(T *&out, size_t count)
    {
        void *q = nullptr;
        const hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) { p.push_back(q); out = (T *)q; }
        return e;
    }
    ~Scratch()
    {
        for (void *q : p) (void)hipFree(q);
    }
};

template <class S, class B>
int build(const uint8_t *ref, int64_t len, bsw::GpuIndex *out)
{
    const int64_t n = 2 * len, N = n + 1;
    Scratch X;
    hipStream_t st = nullptr;                          // the null stream of this device: blocking
    uint8_t *d_ref, *T;
    FB_TRY(X.get(d_ref, (size_t)len));
    FB_TRY(X.get(T, (size_t)n));
    FB_TRY(hipMemcpy(d_ref, ref, (size_t)len, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_make_text, dim3(stride_grid(len)), dim3(256), 0, st, d_ref, len, T);
    FB_TRY(hipGetLastError());
    // 2. buckets
    unsigned long long *d_cnt, *d_cur;
    FB_TRY(X.get(d_cnt, kBuckets));
    FB_TRY(X.get(d_cur, kBuckets));
    FB_TRY(hipMemset(d_cnt, 0, kBuckets * sizeof(unsigned long long)));
    hipLaunchKernelGGL(k_hist, dim3(4096), dim3(256), 0, st, T, n, d_cnt);
    FB_TRY(hipGetLastError());
    unsigned long long h_cnt[kBuckets], h_off[kBuckets + 1];
    FB_TRY(hipMemcpy(h_cnt, d_cnt, sizeof(h_cnt), hipMemcpyDeviceToHost));
    h_off[0] = 0;
    uint64_t maxb = 0;
    for (int k = 0; k < kBuckets; ++k) {
        h_off[k + 1] = h_off[k] + h_cnt[k];
        maxb = std::max<uint64_t>(maxb, h_cnt[k]);
    }
    if ((int64_t)h_off[kBuckets] != N || maxb >= (1ull << 31)) return BSW_E_RANGE;
    FB_TRY(hipMemcpy(d_cur, h_off, sizeof(unsigned long long) * kBuckets, hipMemcpyHostToDevice));
    S *sa = nullptr;
    FB_TRY(hipMalloc(&sa, (size_t)N * sizeof(S)));
    out->d_sa = sa;                                    // owned by the index from here on
    const int64_t per_block = 1 << 16;
    hipLaunchKernelGGL(k_scatter<S>, dim3(grid_of(N, (int)per_block)), dim3(256), 0, st, T, n, per_block, d_cur, sa);
    FB_TRY(hipGetLastError());
    // 3. per-bucket radix sort of 27-base keys
    uint64_t *k_in, *k_out;
    S *v_out;
    FB_TRY(X.get(k_in, maxb));
    FB_TRY(X.get(k_out, maxb));
    FB_TRY(X.get(v_out, maxb));
    size_t tmp_bytes = 0;
    FB_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k_in, k_out, sa, v_out, (int)maxb, 0, 63, st));
    uint8_t *tmp;
    FB_TRY(X.get(tmp, tmp_bytes));
    const int64_t gcap = std::max<int64_t>(1024, (int64_t)maxb / 2);
    int64_t *d_grp;
    unsigned long long *d_ng;
    FB_TRY(X.get(d_grp, 2 * (size_t)gcap));
    FB_TRY(X.get(d_ng, 1));
    std::vector<uint8_t> hT;                           // host text, only for large tie groups
    for (int b = 0; b < kBuckets; ++b) {
        const int64_t m = (int64_t)h_cnt[b], off = (int64_t)h_off[b];
        if (m < 2) continue;
        S *pos = sa + off;
        hipLaunchKernelGGL(k_keys<S>, dim3(grid_of(m)), dim3(256), 0, st, T, n, pos, m, k_in);
        FB_TRY(hipGetLastError());
        size_t tb = tmp_bytes;
        FB_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k_in, k_out, pos, v_out, (int)m, 0, 63, st));
        FB_TRY(hipMemcpy(pos, v_out, (size_t)m * sizeof(S), hipMemcpyDeviceToDevice));
        // 4. tie groups
        FB_TRY(hipMemset(d_ng, 0, sizeof(unsigned long long)));
        hipLaunchKernelGGL(k_ties, dim3(grid_of(m)), dim3(256), 0, st, k_out, m, d_grp, gcap, d_ng);
        FB_TRY(hipGetLastError());
        unsigned long long ng = 0;
        FB_TRY(hipMemcpy(&ng, d_ng, sizeof(ng), hipMemcpyDeviceToHost));
        if (ng == 0) continue;
        if ((int64_t)ng > gcap) return BSW_E_RANGE;
        out->tie_groups += (int64_t)ng;
        hipLaunchKernelGGL(k_sort_small_groups<S>, dim3(grid_of((int64_t)ng)), dim3(256), 0, st, T, n, pos, d_grp,
                           (int64_t)ng);
        FB_TRY(hipGetLastError());
        std::vector<int64_t> g(2 * ng);
        FB_TRY(hipMemcpy(g.data(), d_grp, g.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
        for (unsigned long long q = 0; q < ng; ++q) {
            const int64_t a = g[2 * q], e = g[2 * q + 1];
            if (e - a <= 32) continue;
            if (hT.empty()) {
                hT.resize((size_t)n);
                FB_TRY(hipMemcpy(hT.data(), T, (size_t)n, hipMemcpyDeviceToHost));
            }
            std::vector<S> v((size_t)(e - a));
            FB_TRY(hipMemcpy(v.data(), pos + a, v.size() * sizeof(S), hipMemcpyDeviceToHost));
            std::sort(v.begin(), v.end(), [&](S x, S y) { return suffix_less(hT.data(), n, (int64_t)x, (int64_t)y, 27); });
            FB_TRY(hipMemcpy(pos + a, v.data(), v.size() * sizeof(S), hipMemcpyHostToDevice));
        }
    }
    // 5. BWT, sentinel, occurrence blocks
    uint8_t *bwt = nullptr;
    FB_TRY(hipMalloc(&bwt, (size_t)N));
    out->d_bwt = bwt;
    unsigned long long *d_sent;
    FB_TRY(X.get(d_sent, 1));
    hipLaunchKernelGGL(k_bwt<S>, dim3(stride_grid(N)), dim3(256), 0, st, T, sa, N, bwt, d_sent);
    FB_TRY(hipGetLastError());
    const int64_t nb = (N >> 6) + 1;                   // covers row N (= k + s at most)
    B *blk = nullptr;
    FB_TRY(hipMalloc(&blk, (size_t)nb * sizeof(B)));
    out->d_blk = blk;
    unsigned long long *bc, *pre;
    FB_TRY(X.get(bc, 4 * (size_t)nb));
    FB_TRY(X.get(pre, 4 * (size_t)nb + 1));
    hipLaunchKernelGGL(k_blocks<B>, dim3(grid_of(nb)), dim3(256), 0, st, bwt, N, nb, blk, bc);
    FB_TRY(hipGetLastError());
    size_t sb = 0;
    FB_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, sb, bc, pre, (int)nb, st));
    uint8_t *stmp;
    FB_TRY(X.get(stmp, sb));
    int64_t tot[4];
    for (int c = 0; c < 4; ++c) {
        size_t b2 = sb;
        FB_TRY(hipcub::DeviceScan::ExclusiveSum(stmp, b2, bc + c * nb, pre + c * nb, (int)nb, st));
        unsigned long long last_pre = 0, last_cnt = 0;
        FB_TRY(hipMemcpy(&last_pre, pre + c * nb + nb - 1, sizeof(last_pre), hipMemcpyDeviceToHost));
        FB_TRY(hipMemcpy(&last_cnt, bc + c * nb + nb - 1, sizeof(last_cnt), hipMemcpyDeviceToHost));
        tot[c] = (int64_t)(last_pre + last_cnt);
    }
    hipLaunchKernelGGL(k_block_counts<B>, dim3(grid_of(nb)), dim3(256), 0, st, nb, pre, blk);
    FB_TRY(hipGetLastError());
    unsigned long long sent = 0;
    FB_TRY(hipMemcpy(&sent, d_sent, sizeof(sent), hipMemcpyDeviceToHost));
    FB_TRY(hipDeviceSynchronize());
    out->n = n;
    out->sentinel = (int64_t)sent;
    out->count[0] = 1;
    for (int c = 0; c < 4; ++c) out->count[c + 1] = out->count[c] + tot[c];
    return BSW_OK;
}

}  // namespace

int bsw::fmi_check_gpu(int device, bool wide, const void *d_sa, const uint8_t *d_bwt, const void *d_blk, int64_t n,
                       const int64_t *count, int64_t *bad)
{
    *bad = -1;
    if (hipSetDevice(device) != hipSuccess) return BSW_E_HIP;
    const int64_t N = n + 1, nb = (N >> 6) + 1;
    Scratch X;
    int64_t *d_count;
    unsigned int *seen;
    unsigned long long *d_bad;
    FB_TRY(X.get(d_count, 5));
    FB_TRY(X.get(seen, (size_t)(N + 31) / 32));
    FB_TRY(X.get(d_bad, 1));
    FB_TRY(hipMemcpy(d_count, count, 5 * sizeof(int64_t), hipMemcpyHostToDevice));
    FB_TRY(hipMemset(seen, 0, (size_t)(N + 31) / 32 * sizeof(unsigned int)));
    FB_TRY(hipMemset(d_bad, 0, sizeof(unsigned long long)));
    if (wide) {
        hipLaunchKernelGGL(k_chk_blocks<FmiBlockW>, dim3(grid_of(nb)), dim3(256), 0, 0, (const FmiBlockW *)d_blk, nb,
                           d_count, d_bad);
        hipLaunchKernelGGL((k_chk_lf<uint64_t, FmiBlockW>), dim3(stride_grid(N)), dim3(256), 0, 0, (const uint64_t *)d_sa,
                           d_bwt, (const FmiBlockW *)d_blk, N, d_count, seen, d_bad);
    } else {
        hipLaunchKernelGGL(k_chk_blocks<FmiBlock>, dim3(grid_of(nb)), dim3(256), 0, 0, (const FmiBlock *)d_blk, nb,
                           d_count, d_bad);
        hipLaunchKernelGGL((k_chk_lf<uint32_t, FmiBlock>), dim3(stride_grid(N)), dim3(256), 0, 0, (const uint32_t *)d_sa,
                           d_bwt, (const FmiBlock *)d_blk, N, d_count, seen, d_bad);
    }
    FB_TRY(hipGetLastError());
    unsigned long long b = 0;
    FB_TRY(hipMemcpy(&b, d_bad, sizeof(b), hipMemcpyDeviceToHost));
    *bad = (int64_t)b;
    return BSW_OK;
}

int bsw::fmi_build_gpu(const uint8_t *ref, int64_t ref_len, int device, bool wide, GpuIndex *out)
{
    *out = GpuIndex{};
    if (hipSetDevice(device) != hipSuccess) return BSW_E_HIP;
    const int rc = wide ? build<uint64_t, FmiBlockW>(ref, ref_len, out) : build<uint32_t, FmiBlock>(ref, ref_len, out);
    if (rc) {
        if (out->d_sa) (void)hipFree(out->d_sa);
        if (out->d_bwt) (void)hipFree(out->d_bwt);
        if (out->d_blk) (void)hipFree(out->d_blk);
        *out = GpuIndex{};
    }
    return rc;
}
