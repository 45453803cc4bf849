// bsw_memchain.hip -- seeds -> chains on the GPU: bwa's mem_chain + mem_chain_flt per read
// (include/bsw_fmi.h bsw_mem_chain_device).  Oracle: oracle/chain_ref.c.
//
// Work per read is a short, branchy, sequential walk (a handful of intervals, a sorted chain
// list, a weight sort), so the mapping is one thread per read over per-read regions of flat
// HBM scratch, sized exactly by a counting pass:
//   k_count   raw seeds per read = sum over its intervals of min(max_occ, ceil(s / step))
//   (hipcub exclusive scan -> each read's region [off, off + cnt))
//   k_chain   SA lookups, test_and_merge against the chain list kept sorted by start (a
//             single-leaf kbtree: lower = the first chain of equal start, else the last smaller
//             one; a new chain goes right after the first chain of equal start), the chains'
//             seeds as linked lists in a seed pool, chain weights, klib's ks_introsort by
//             weight (upstream's tie order), the flt overlap / drop / kept rules; leaves the
//             kept chains' order and the read's kept seed count
//   (hipcub exclusive scan of the kept counts -> output offsets; the total comes back)
//   k_emit    kept chains' seeds -> compact (seeds, seed_read, seed_chain), chain order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <algorithm>
#include "../../include/bsw_fmi.h"
#include "bsw_fmi_internal.h"
#include "bsw_devcache.h"

namespace {

struct COpt {
    int32_t max_occ, w, max_chain_gap, min_chain_weight, min_seed_len, max_chain_extend;
    float drop_ratio, mask_level;
};

struct PoolSeed {                     // one seed of a chain (the chain's list: next[])
    int64_t rbeg;
    int32_t qbeg, len;
};

struct ChainRec {
    int64_t pos;                      // start = the first seed's rbeg
    int32_t head, tail, n;            // seed list in the pool (insertion order)
    int32_t w, kept, first;           // mem_chain_flt state
};

struct WI {                           // introsort element: weight and chain index
    int32_t w, idx;
};

__device__ __forceinline__ int64_t n_taken(uint64_t s, int max_occ)
{
    const uint64_t step = s > (uint64_t)max_occ ? s / (uint64_t)max_occ : 1;
    const uint64_t n = (s + step - 1) / step;          // k = 0, step, ... < s
    return (int64_t)(n < (uint64_t)max_occ ? n : (uint64_t)max_occ);
}

__global__ void k_count(COpt o, const int32_t *__restrict__ read_len, int32_t n_reads,
                        const bsw_bwtintv_t *__restrict__ mems, int32_t cap, const int32_t *__restrict__ n_mems,
                        int64_t *__restrict__ cnt)
{
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_reads) return;
    int64_t c = 0;
    if (read_len[r] >= o.min_seed_len) {
        const int nm = min(n_mems[r], cap);
        for (int t = 0; t < nm; ++t) c += n_taken(mems[(int64_t)r * cap + t].x[2], o.max_occ);
    }
    cnt[r] = c;
}

// ---- klib ksort.h on WI with lt(a, b) = a.w > b.w (mem_chain_flt's flt_lt)
__device__ __forceinline__ bool wlt(const WI &a, const WI &b) { return a.w > b.w; }

__device__ void w_insertsort(WI *s, WI *t)
{
    for (WI *i = s + 1; i < t; ++i)
        for (WI *j = i; j > s && wlt(*j, *(j - 1)); --j) {
            const WI x = *j; *j = *(j - 1); *(j - 1) = x;
        }
}

__device__ void w_combsort(size_t n, WI *a)
{
    const double shrink_factor = 1.2473309501039786540366528676643;
    int do_swap;
    size_t gap = n;
    do {
        if (gap > 2) {
            gap = (size_t)(gap / shrink_factor);
            if (gap == 9 || gap == 10) gap = 11;
        }
        do_swap = 0;
        for (WI *i = a; i < a + n - gap; ++i) {
            WI *j = i + gap;
            if (wlt(*j, *i)) {
                const WI x = *i; *i = *j; *j = x;
                do_swap = 1;
            }
        }
    } while (do_swap || gap > 2);
    if (gap != 1) w_insertsort(a, a + n);
}

__device__ void w_introsort(size_t n, WI *a)
{
    struct Frame { WI *left, *right; int depth; };
    Frame stack[2 * 64 + 2];                            // (sizeof(size_t) * d + 2) for n < 2^64
    int d;
    if (n < 1) return;
    if (n == 2) {
        if (wlt(a[1], a[0])) { const WI x = a[0]; a[0] = a[1]; a[1] = x; }
        return;
    }
    for (d = 2; 1ul << d < n; ++d) ;
    Frame *top = stack;
    WI *s = a, *t = a + (n - 1), *i, *j, *k;
    d <<= 1;
    while (true) {
        if (s < t) {
            if (--d == 0) {
                w_combsort((size_t)(t - s + 1), s);
                t = s;
                continue;
            }
            i = s; j = t; k = i + ((j - i) >> 1) + 1;
            if (wlt(*k, *i)) {
                if (wlt(*k, *j)) k = j;
            } else {
                k = wlt(*j, *i) ? i : j;
            }
            const WI rp = *k;
            if (k != t) { const WI x = *k; *k = *t; *t = x; }
            for (;;) {
                do ++i; while (wlt(*i, rp));
                do --j; while (i <= j && wlt(rp, *j));
                if (j <= i) break;
                const WI x = *i; *i = *j; *j = x;
            }
            { const WI x = *i; *i = *t; *t = x; }
            if (i - s > t - i) {
                if (i - s > 16) { top->left = s; top->right = i - 1; top->depth = d; ++top; }
                s = t - i > 16 ? i + 1 : t;
            } else {
                if (t - i > 16) { top->left = i + 1; top->right = t; top->depth = d; ++top; }
                t = i - s > 16 ? i - 1 : s;
            }
        } else {
            if (top == stack) {
                w_insertsort(a, a + n);
                return;
            }
            --top; s = top->left; t = top->right; d = top->depth;
        }
    }
}

// test_and_merge: 1 = absorbed (appended to c, or contained)
__device__ bool test_and_merge(const COpt &o, int64_t l_pac, ChainRec &c, PoolSeed *pool, int32_t *next,
                               int32_t &np, const PoolSeed &p)
{
    const PoolSeed f = pool[c.head], last = pool[c.tail];
    const int64_t qend = last.qbeg + last.len, rend = last.rbeg + last.len;
    if (p.qbeg >= f.qbeg && p.qbeg + p.len <= qend && p.rbeg >= f.rbeg && p.rbeg + p.len <= rend) return true;
    if ((last.rbeg < l_pac || f.rbeg < l_pac) && p.rbeg >= l_pac) return false;
    const int64_t x = p.qbeg - last.qbeg, y = p.rbeg - last.rbeg;
    if (y >= 0 && x - y <= o.w && y - x <= o.w && x - last.len < o.max_chain_gap && y - last.len < o.max_chain_gap) {
        pool[np] = p;
        next[np] = -1;
        next[c.tail] = np;
        c.tail = np++;
        c.n++;
        return true;
    }
    return false;
}

__device__ int chain_weight(const ChainRec &c, const PoolSeed *pool, const int32_t *next)
{
    int64_t end = 0;
    int w = 0, tmp;
    for (int32_t k = c.head; k >= 0; k = next[k]) {
        const PoolSeed s = pool[k];
        if (s.qbeg >= end) w += s.len;
        else if (s.qbeg + s.len > end) w += (int)(s.qbeg + s.len - end);
        end = max(end, (int64_t)s.qbeg + s.len);
    }
    tmp = w; w = 0; end = 0;
    for (int32_t k = c.head; k >= 0; k = next[k]) {
        const PoolSeed s = pool[k];
        if (s.rbeg >= end) w += s.len;
        else if (s.rbeg + s.len > end) w += (int)(s.rbeg + s.len - end);
        end = max(end, s.rbeg + s.len);
    }
    w = min(w, tmp);
    return w < (1 << 30) ? w : (1 << 30) - 1;
}

// per read: region [off, off + cnt) of pool / next / chains / order / wi / list
template <class S>
__global__ void k_chain(COpt o, const S *__restrict__ sa, int64_t l_pac, const int32_t *__restrict__ read_len,
                        int32_t n_reads, const bsw_bwtintv_t *__restrict__ mems, int32_t cap,
                        const int32_t *__restrict__ n_mems, const int64_t *__restrict__ off,
                        PoolSeed *__restrict__ pool_all, int32_t *__restrict__ next_all,
                        ChainRec *__restrict__ chains_all, int32_t *__restrict__ ord_all, WI *__restrict__ wi_all,
                        int32_t *__restrict__ list_all, int32_t *__restrict__ n_kept, int64_t *__restrict__ kcnt)
{
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_reads) return;
    const int64_t base = off[r];
    PoolSeed *pool = pool_all + base;
    int32_t *next = next_all + base, *ord = ord_all + base, *list = list_all + base;
    ChainRec *ch = chains_all + base;
    WI *wi = wi_all + base;
    int32_t np = 0, nc = 0;                             // pool seeds, chains (ord[0 .. nc) by start)
    if (read_len[r] >= o.min_seed_len) {
        const int nm = min(n_mems[r], cap);
        for (int t = 0; t < nm; ++t) {
            const bsw_bwtintv_t p = mems[(int64_t)r * cap + t];
            const int slen = (int)((uint32_t)p.info - (uint32_t)(p.info >> 32));
            const uint64_t step = p.x[2] > (uint64_t)o.max_occ ? p.x[2] / (uint64_t)o.max_occ : 1;
            uint64_t k = 0;
            for (int count = 0; k < p.x[2] && count < o.max_occ; k += step, ++count) {
                PoolSeed s;
                s.rbeg = (int64_t)sa[p.x[0] + k];
                s.qbeg = (int32_t)(p.info >> 32);
                s.len = slen;
                if (s.rbeg < l_pac && l_pac < s.rbeg + s.len) continue;      // bridging: rid < 0
                int lo = 0, hi = nc;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (ch[ord[mid]].pos < s.rbeg) lo = mid + 1; else hi = mid;
                }
                const bool eq = lo < nc && ch[ord[lo]].pos == s.rbeg;
                const int lower = eq ? lo : lo - 1;
                if (lower >= 0 && test_and_merge(o, l_pac, ch[ord[lower]], pool, next, np, s)) continue;
                const int at = eq ? lo + 1 : lo;
                for (int u = nc; u > at; --u) ord[u] = ord[u - 1];
                ChainRec c;
                c.pos = s.rbeg;
                c.head = c.tail = np;
                c.n = 1;
                c.w = c.kept = 0;
                c.first = -1;
                pool[np] = s;
                next[np] = -1;
                ++np;
                ch[nc] = c;
                ord[at] = nc;
                ++nc;
            }
        }
    }
    // mem_chain_flt over a[] = chains in start order (wi: weight, chain index)
    int n_chn = 0;
    for (int i = 0; i < nc; ++i) {
        ChainRec &c = ch[ord[i]];
        c.first = -1;
        c.kept = 0;
        c.w = chain_weight(c, pool, next);
        if (c.w >= o.min_chain_weight) wi[n_chn++] = WI{c.w, ord[i]};
    }
    int nk = 0;
    if (n_chn > 0) {
        w_introsort((size_t)n_chn, wi);
        // list[] holds indices into wi of the kept non-shadowed chains ("chains" kvec)
        int nch = 0;
        ch[wi[0].idx].kept = 3;
        list[nch++] = 0;
        for (int i = 1; i < n_chn; ++i) {
            ChainRec &ci = ch[wi[i].idx];
            const PoolSeed bi = pool[ci.head], ei = pool[ci.tail];
            const int beg_i = bi.qbeg, end_i = ei.qbeg + ei.len;
            int large_ovlp = 0, k;
            for (k = 0; k < nch; ++k) {
                const int j = list[k];
                ChainRec &cj = ch[wi[j].idx];
                const PoolSeed bj = pool[cj.head], ej = pool[cj.tail];
                const int beg_j = bj.qbeg, end_j = ej.qbeg + ej.len;
                const int b_max = max(beg_j, beg_i), e_min = min(end_j, end_i);
                if (e_min > b_max) {
                    const int li = end_i - beg_i, lj = end_j - beg_j;
                    const int min_l = min(li, lj);
                    if (e_min - b_max >= min_l * o.mask_level && min_l < o.max_chain_gap) {
                        large_ovlp = 1;
                        if (cj.first < 0) cj.first = i;
                        if (ci.w < cj.w * o.drop_ratio && cj.w - ci.w >= o.min_seed_len << 1) break;
                    }
                }
            }
            if (k == nch) {
                list[nch++] = i;
                ci.kept = large_ovlp ? 2 : 3;
            }
        }
        for (int i = 0; i < nch; ++i) {
            const ChainRec &c = ch[wi[list[i]].idx];
            if (c.first >= 0) ch[wi[c.first].idx].kept = 1;
        }
        int i, k;
        for (i = k = 0; i < n_chn; ++i) {
            const int kp = ch[wi[i].idx].kept;
            if (kp == 0 || kp == 3) continue;
            if (++k >= o.max_chain_extend) break;
        }
        for (; i < n_chn; ++i)
            if (ch[wi[i].idx].kept < 3) ch[wi[i].idx].kept = 0;
        int64_t ks = 0;
        for (i = 0; i < n_chn; ++i) {
            const ChainRec &c = ch[wi[i].idx];
            if (c.kept == 0) continue;
            ord[nk++] = wi[i].idx;                      // the kept chains, in processing order
            ks += c.n;
        }
        kcnt[r] = ks;
    } else {
        kcnt[r] = 0;
    }
    n_kept[r] = nk;
}

__global__ void k_emit(int32_t n_reads, const int64_t *__restrict__ off, const PoolSeed *__restrict__ pool_all,
                       const int32_t *__restrict__ next_all, const ChainRec *__restrict__ chains_all,
                       const int32_t *__restrict__ ord_all, const int32_t *__restrict__ n_kept,
                       const int64_t *__restrict__ out_off, int64_t seed_cap, bsw_seed_t *__restrict__ seeds,
                       int32_t *__restrict__ seed_read, int32_t *__restrict__ seed_chain)
{
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_reads) return;
    const int64_t base = off[r];
    const PoolSeed *pool = pool_all + base;
    const int32_t *next = next_all + base, *ord = ord_all + base;
    const ChainRec *ch = chains_all + base;
    int64_t o = out_off[r];
    for (int c = 0; c < n_kept[r]; ++c)
        for (int32_t k = ch[ord[c]].head; k >= 0; k = next[k], ++o) {
            if (o >= seed_cap) return;
            const PoolSeed s = pool[k];
            seeds[o] = bsw_seed_t{s.rbeg, s.qbeg, s.len};
            seed_read[o] = r;
            seed_chain[o] = c;
        }
}

int hip_rc(hipError_t e) { return e == hipSuccess ? BSW_OK : (e == hipErrorOutOfMemory ? BSW_E_NOMEM : BSW_E_HIP); }

#define MC_TRY(x)                                          \
    do {                                                   \
        const int rc_ = hip_rc(x);                         \
        if (rc_) return rc_;                               \
    } while (0)

using bsw::CachedBufs;

int run_chain(const bsw::FmiView &f, const COpt &o, const int32_t *d_len, int32_t n, const bsw_bwtintv_t *d_mems,
              int32_t cap, const int32_t *d_nm, bsw_seed_t *d_seeds, int32_t *d_sr, int32_t *d_sc, int64_t seed_cap,
              int64_t *n_seeds, hipStream_t s)
{
    CachedBufs B(f.device);
    B.stream = s;
    int64_t *cnt, *off, *kcnt, *koff;
    int32_t *n_kept;
    MC_TRY(B.get(cnt, (size_t)n + 1));
    MC_TRY(B.get(off, (size_t)n + 1));
    MC_TRY(B.get(kcnt, (size_t)n + 1));
    MC_TRY(B.get(koff, (size_t)n + 1));
    MC_TRY(B.get(n_kept, (size_t)n));
    const dim3 g((unsigned)((n + 63) / 64)), b(64);
    hipLaunchKernelGGL(k_count, g, b, 0, s, o, d_len, n, d_mems, cap, d_nm, cnt);
    MC_TRY(hipGetLastError());
    MC_TRY(hipMemsetAsync(cnt + n, 0, sizeof(int64_t), s));
    size_t tb = 0, tb2 = 0;
    MC_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, off, n + 1, s));
    MC_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, kcnt, koff, n + 1, s));
    uint8_t *tmp = nullptr;
    MC_TRY(B.get(tmp, std::max(tb, tb2)));
    MC_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, off, n + 1, s));
    int64_t raw = 0;
    MC_TRY(hipMemcpyAsync(&raw, off + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    MC_TRY(hipStreamSynchronize(s));
    PoolSeed *pool;
    int32_t *next, *ord, *list;
    ChainRec *chains;
    WI *wi;
    const size_t R = (size_t)std::max<int64_t>(raw, 1);
    MC_TRY(B.get(pool, R));
    MC_TRY(B.get(next, R));
    MC_TRY(B.get(chains, R));
    MC_TRY(B.get(ord, R));
    MC_TRY(B.get(wi, R));
    MC_TRY(B.get(list, R));
    if (f.sa64)
        hipLaunchKernelGGL(k_chain<uint64_t>, g, b, 0, s, o, (const uint64_t *)f.d_sa, f.l_pac, d_len, n, d_mems, cap,
                           d_nm, off, pool, next, chains, ord, wi, list, n_kept, kcnt);
    else
        hipLaunchKernelGGL(k_chain<uint32_t>, g, b, 0, s, o, (const uint32_t *)f.d_sa, f.l_pac, d_len, n, d_mems, cap,
                           d_nm, off, pool, next, chains, ord, wi, list, n_kept, kcnt);
    MC_TRY(hipGetLastError());
    MC_TRY(hipMemsetAsync(kcnt + n, 0, sizeof(int64_t), s));
    MC_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, kcnt, koff, n + 1, s));
    int64_t total = 0;
    MC_TRY(hipMemcpyAsync(&total, koff + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    MC_TRY(hipStreamSynchronize(s));
    *n_seeds = total;
    if (total > seed_cap) return BSW_E_RANGE;
    if (total > 0) {
        hipLaunchKernelGGL(k_emit, g, b, 0, s, n, off, pool, next, chains, ord, n_kept, koff, seed_cap, d_seeds, d_sr,
                           d_sc);
        MC_TRY(hipGetLastError());
    }
    MC_TRY(hipStreamSynchronize(s));
    return BSW_OK;
}

}  // namespace

extern "C" void bsw_chain_opt_default(bsw_chain_opt_t *opt)
{
    opt->max_occ = 500;
    opt->w = 100;
    opt->max_chain_gap = 10000;
    opt->min_chain_weight = 0;
    opt->min_seed_len = 19;
    opt->max_chain_extend = 1 << 30;
    opt->drop_ratio = 0.5f;
    opt->mask_level = 0.5f;
}

extern "C" int bsw_mem_chain_device(bsw_fmi_t *fmi, const bsw_chain_opt_t *opt, const int32_t *d_read_len,
                                    int32_t n_reads, const bsw_bwtintv_t *d_mems, int32_t cap,
                                    const int32_t *d_n_mems, bsw_seed_t *d_seeds, int32_t *d_seed_read,
                                    int32_t *d_seed_chain, int64_t seed_cap, int64_t *n_seeds, void *stream)
{
    if (!fmi || !opt || !n_seeds || n_reads < 0 || cap < 0 || seed_cap < 0) return BSW_E_INVAL;
    if (opt->max_occ < 1 || opt->w < 0 || opt->max_chain_gap < 0 || opt->max_chain_extend < 0) return BSW_E_INVAL;
    *n_seeds = 0;
    if (n_reads == 0) return BSW_OK;
    if (!d_read_len || !d_n_mems || (cap > 0 && !d_mems) || (seed_cap > 0 && (!d_seeds || !d_seed_read || !d_seed_chain)))
        return BSW_E_INVAL;
    bsw::FmiView f;
    if (const int rc = bsw::fmi_view(fmi, &f)) return rc;
    std::lock_guard<std::mutex> lk(*f.mu);
    if (hipSetDevice(f.device) != hipSuccess) return BSW_E_HIP;
    COpt o{opt->max_occ, opt->w, opt->max_chain_gap, opt->min_chain_weight, opt->min_seed_len, opt->max_chain_extend,
           opt->drop_ratio, opt->mask_level};
    return run_chain(f, o, d_read_len, n_reads, d_mems, cap, d_n_mems, d_seeds, d_seed_read, d_seed_chain, seed_cap,
                     n_seeds, stream ? (hipStream_t)stream : f.stream);
}
