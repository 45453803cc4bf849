// bsw_chain.hip -- mem_chain2aln over chains with every per-read decision on the GPU
// (include/bsw_ext.h bsw_chain2aln_device / bsw_chain2aln_resident).
//
// Same semantics as chain_rounds in bsw_ext.cpp (oracle: oracle/ext_ref.c oracle_chain2aln):
// per read, chains in order and each chain's seeds by score descending (ties: the later seed
// first); a seed lying around the diagonal of an already extended region of its read is
// skipped unless an extended seed of its own chain, >= 95% as long, overlaps it by >= 1/4 of
// its length on another diagonal.  Work runs in rounds batched across reads: round r extends,
// for every read, the next seed its containment test keeps.  Here one thread per read runs the
// per-read order (k_prep), the containment scan and the pick (k_pick, jobs compacted by a
// wave-aggregated counter), the round's LEFT / RIGHT extensions go through the device
// extension pipeline (bsw_extend_seeds_device), and k_scatter files the regions; the host only
// reads back one job count per round.  Job order inside a round is whatever the counter hands
// out: jobs are independent and results are filed by seed index, so outputs are deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include "../../include/bsw_ext.h"
#include "bsw_internal.h"
#include "bsw_devcache.h"

namespace {

struct ChainParams {
    int32_t o_del, e_del, o_ins, e_ins, a, w;
    int64_t ref_len, l_pac;
};

__device__ __forceinline__ int d_cal_max_gap(const ChainParams &p, int qlen)
{
    const int l_del = (int)((double)(qlen * p.a - p.o_del) / p.e_del + 1.);
    const int l_ins = (int)((double)(qlen * p.a - p.o_ins) / p.e_ins + 1.);
    int l = max(l_del, l_ins);
    l = max(l, 1);
    return min(l, p.w << 1);
}

// upstream's "seed contained in an earlier region of the read" test
__device__ bool d_contained(const ChainParams &p, const bsw_seed_t &s, int l_query, const bsw_alnreg_t *out,
                            const int32_t *av, int32_t nav)
{
    for (int32_t k = 0; k < nav; ++k) {
        const bsw_alnreg_t q = out[av[k]];
        if (s.rbeg < q.rb || s.rbeg + s.len > q.re || s.qbeg < q.qb || s.qbeg + s.len > q.qe) continue;
        if (s.len - q.seedlen0 > .1 * l_query) continue;
        int qd = s.qbeg - q.qb;
        int64_t rd = s.rbeg - q.rb;
        int max_gap = d_cal_max_gap(p, qd < rd ? qd : (int)rd);
        int w = min(max_gap, q.w);
        if (qd - rd < w && rd - qd < w) return true;
        qd = q.qe - (s.qbeg + s.len);
        rd = q.re - (s.rbeg + s.len);
        max_gap = d_cal_max_gap(p, qd < rd ? qd : (int)rd);
        w = min(max_gap, q.w);
        if (qd - rd < w && rd - qd < w) return true;
    }
    return false;
}

// seed runs per read: sbeg[r], send[r] (memset 0 first); err |= 1 on a bad or unsorted read id
__global__ void k_runs(const int32_t *__restrict__ sr, int32_t ns, int32_t n_reads, int32_t *__restrict__ sbeg,
                       int32_t *__restrict__ send, int32_t *__restrict__ err)
{
    const int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ns) return;
    const int32_t r = sr[k];
    if (r < 0 || r >= n_reads || (k > 0 && sr[k - 1] > r)) {
        atomicOr(err, 1);
        return;
    }
    if (k == 0 || sr[k - 1] != r) sbeg[r] = k;
    if (k == ns - 1 || sr[k + 1] != r) send[r] = k + 1;
}

// per read: regions zeroed, chain order (insertion sort of each chain: score desc, index desc)
// and each chain's target window (mem_chain2aln's rmax[]: min / max of its seeds' reach, clipped
// to the reference, the first seed's side of l_pac) at cwin[2 * head]
__global__ void k_prep(int32_t n_reads, const int32_t *__restrict__ sbeg, const int32_t *__restrict__ send,
                       const bsw_seed_t *__restrict__ seeds, const int32_t *__restrict__ sc,
                       const int32_t *__restrict__ read_len, const ChainParams p, int32_t *__restrict__ order,
                       int32_t *__restrict__ chain_of, int64_t *__restrict__ cwin, int32_t *__restrict__ pos,
                       int32_t *__restrict__ nav, bsw_alnreg_t *__restrict__ out, int32_t *__restrict__ ext)
{
    const int32_t a = p.a;
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_reads) return;
    const int32_t b = sbeg[r], e = send[r];
    bsw_alnreg_t z;
    memset(&z, 0, sizeof(z));
    for (int32_t k = b; k < e; ++k) {
        out[k] = z;
        ext[k] = 0;
    }
    for (int32_t c0 = b; c0 < e;) {
        int32_t c1 = c0;
        const int32_t cid = sc[c0];
        while (c1 < e && sc[c1] == cid) ++c1;
        const int l_query = read_len[r];
        int64_t lo = p.ref_len, hi = 0, first = -1;
        for (int32_t i = c0; i < c1; ++i) {
            const bsw_seed_t t = seeds[i];
            if (t.len <= 0) continue;
            if (first < 0) first = t.rbeg;
            const int qe = t.qbeg + t.len;
            lo = min(lo, t.rbeg - (int64_t)(t.qbeg + d_cal_max_gap(p, t.qbeg)));
            hi = max(hi, t.rbeg + t.len + (int64_t)((l_query - qe) + d_cal_max_gap(p, l_query - qe)));
        }
        lo = max(lo, (int64_t)0);
        hi = min(hi, p.ref_len);
        if (p.l_pac > 0 && lo < p.l_pac && p.l_pac < hi) {
            if (first < p.l_pac) hi = p.l_pac;
            else lo = p.l_pac;
        }
        cwin[2 * (int64_t)c0] = lo;
        cwin[2 * (int64_t)c0 + 1] = hi;
        for (int32_t i = c0; i < c1; ++i) {
            chain_of[i] = c0;
            // insert i into order[c0 .. i): (len * a, index) descending
            const int64_t ki = (int64_t)seeds[i].len * a;
            int32_t j = i;
            while (j > c0) {
                const int32_t x = order[j - 1];
                const int64_t kx = (int64_t)seeds[x].len * a;
                if (kx > ki || (kx == ki && x > i)) break;
                order[j] = x;
                --j;
            }
            order[j] = i;
        }
        c0 = c1;
    }
    pos[r] = b;
    nav[r] = 0;
}

// per read: the next seed its containment test keeps -> one job (wave-aggregated counter)
__global__ __launch_bounds__(64) void k_pick(int32_t n_reads, const int32_t *__restrict__ sbeg,
                                             const int32_t *__restrict__ send, const bsw_seed_t *__restrict__ seeds,
                                             const int64_t *__restrict__ read_off,
                                             const int32_t *__restrict__ read_len, const int32_t *__restrict__ order,
                                             const int32_t *__restrict__ chain_of, const int64_t *__restrict__ cwin,
                                             const int32_t *__restrict__ ext,
                                             const bsw_alnreg_t *__restrict__ out, const int32_t *__restrict__ av,
                                             const int32_t *__restrict__ nav, int32_t *__restrict__ pos,
                                             const ChainParams p, int32_t *__restrict__ cnt,
                                             int32_t *__restrict__ jsi, int32_t *__restrict__ jrun,
                                             int64_t *__restrict__ joff, int32_t *__restrict__ jlen,
                                             bsw_seed_t *__restrict__ jseed, int64_t *__restrict__ jwin)
{
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    int32_t pick = -1;
    if (r < n_reads) {
        const int32_t b = sbeg[r], e = send[r];
        int32_t ps = pos[r];
        const int l_query = read_len[r];
        while (ps < e) {
            const int32_t si = order[ps++];
            const bsw_seed_t s = seeds[si];
            if (s.len > 0 && d_contained(p, s, l_query, out, av + b, nav[r])) {
                // overlapping extended seeds of the same chain processed earlier
                bool keep = false;
                const int32_t c0 = chain_of[si];
                for (int32_t q = c0; q < ps - 1 && !keep; ++q) {
                    const int32_t ti = order[q];
                    if (!ext[ti]) continue;
                    const bsw_seed_t t = seeds[ti];
                    if (t.len < s.len * .95) continue;
                    if (s.qbeg <= t.qbeg && s.qbeg + s.len - t.qbeg >= s.len >> 2 &&
                        t.qbeg - s.qbeg != t.rbeg - s.rbeg) keep = true;
                    if (t.qbeg <= s.qbeg && t.qbeg + t.len - s.qbeg >= s.len >> 2 &&
                        s.qbeg - t.qbeg != s.rbeg - t.rbeg) keep = true;
                }
                if (!keep) continue;                   // skipped: next seed of this read
            }
            pick = si;
            break;
        }
        pos[r] = ps;
    }
    // compaction: one atomic per wave
    const uint64_t m = __ballot(pick >= 0);
    if (m == 0) return;
    const int lane = (int)__lane_id();
    const int leader = __ffsll((unsigned long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(cnt, __popcll(m));
    base = __shfl(base, leader);
    if (pick >= 0) {
        const int j = base + __popcll(m & ((1ull << lane) - 1));
        jsi[j] = pick;
        jrun[j] = r;
        joff[j] = read_off[r];
        jlen[j] = read_len[r];
        jseed[j] = seeds[pick];
        const int64_t h = chain_of[pick];
        jwin[2 * j] = cwin[2 * h];
        jwin[2 * j + 1] = cwin[2 * h + 1];
    }
}

// file the round's regions: out[si], ext[si], the read's region list
__global__ void k_scatter(int32_t nj, const int32_t *__restrict__ jsi, const int32_t *__restrict__ jrun,
                          const bsw_alnreg_t *__restrict__ jout, const int32_t *__restrict__ sbeg,
                          bsw_alnreg_t *__restrict__ out, int32_t *__restrict__ ext, int32_t *__restrict__ av,
                          int32_t *__restrict__ nav)
{
    const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nj) return;
    const int32_t si = jsi[j], r = jrun[j];
    out[si] = jout[j];
    ext[si] = 1;
    const int32_t k = nav[r];                          // one job per read per round: no race
    av[sbeg[r] + k] = si;
    nav[r] = k + 1;
}

float ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

#define CH_TRY(x)                                                                            \
    do {                                                                                     \
        const hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return e_ == hipErrorOutOfMemory ? BSW_E_NOMEM : BSW_E_HIP;    \
    } while (0)

}  // namespace

namespace bsw {

// The rounds over device-resident inputs (d_*), regions / flags into d_out / d_ext.
int chain_rounds_device(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *d_reads, const int64_t *d_read_off,
                        const int32_t *d_read_len, int32_t n_reads, const bsw_seed_t *d_seeds,
                        const int32_t *d_sr, const int32_t *d_sc, int32_t ns, bsw_alnreg_t *d_out, int32_t *d_ext,
                        bsw_chain_stats_t *cs)
{
    *cs = bsw_chain_stats_t{};
    if (ns == 0) return BSW_OK;
    const int dev = ctx_device(ctx);
    CH_TRY(hipSetDevice(dev));
    bsw_params_t prm;
    ctx_params(ctx, &prm);
    const int64_t ref_len = ctx_refres_len(ctx);
    if (ref_len < 0) return BSW_E_INVAL;                // no resident reference
    if (const int rc = ext_opt_check(opt, ref_len)) return rc;
    ChainParams p{prm.o_del, prm.e_del, prm.o_ins, prm.e_ins, prm.mat[0], opt->w, ref_len, opt->l_pac};
    const auto tp = std::chrono::steady_clock::now();
    // a cached stream + pinned readback words and cached scratch (bsw_devcache.h): no driver
    // allocations per call.  B is destroyed first: it synchronises the stream, then returns its
    // blocks; the lease goes back last
    StreamLease L;
    CH_TRY(stream_lease(dev, L));
    struct LeaseGuard {
        StreamLease &l;
        ~LeaseGuard() { (void)hipStreamSynchronize(l.s); stream_return(l); }
    } lg{L};
    hipStream_t st = L.s;
    int32_t *h = L.h;                                   // pinned readback of the round's job count
    CachedBufs B(dev);
    B.stream = st;
    int32_t *sbeg, *send, *order, *chain_of, *pos, *nav, *av, *cnt, *jsi, *jrun, *jlen, *err;
    int64_t *joff, *cwin, *jwin;
    bsw_seed_t *jseed;
    bsw_alnreg_t *jout;
    const size_t nr = (size_t)n_reads;
    CH_TRY(B.get(sbeg, nr)); CH_TRY(B.get(send, nr)); CH_TRY(B.get(pos, nr)); CH_TRY(B.get(nav, nr));
    CH_TRY(B.get(order, ns)); CH_TRY(B.get(chain_of, ns)); CH_TRY(B.get(av, ns));
    CH_TRY(B.get(cnt, 2)); CH_TRY(B.get(err, 1));
    CH_TRY(B.get(jsi, nr)); CH_TRY(B.get(jrun, nr)); CH_TRY(B.get(jlen, nr)); CH_TRY(B.get(joff, nr));
    CH_TRY(B.get(jseed, nr)); CH_TRY(B.get(jout, nr));
    CH_TRY(B.get(cwin, 2 * (size_t)ns)); CH_TRY(B.get(jwin, 2 * nr));
    CH_TRY(hipMemsetAsync(sbeg, 0, nr * sizeof(int32_t), st));
    CH_TRY(hipMemsetAsync(send, 0, nr * sizeof(int32_t), st));
    CH_TRY(hipMemsetAsync(err, 0, sizeof(int32_t), st));
    hipLaunchKernelGGL(k_runs, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, st, d_sr, ns, n_reads, sbeg, send, err);
    CH_TRY(hipGetLastError());
    CH_TRY(hipMemcpyAsync(h, err, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    CH_TRY(hipStreamSynchronize(st));
    if (h[0]) return BSW_E_INVAL;                       // unsorted / out-of-range seed_read
    const unsigned gr = (unsigned)((nr + 63) / 64);
    hipLaunchKernelGGL(k_prep, dim3(gr), dim3(64), 0, st, n_reads, sbeg, send, d_seeds, d_sc, d_read_len, p, order,
                       chain_of, cwin, pos, nav, d_out, d_ext);
    CH_TRY(hipGetLastError());
    CH_TRY(hipStreamSynchronize(st));
    cs->prep_ms = ms_since(tp);
    for (;;) {
        const auto tc = std::chrono::steady_clock::now();
        CH_TRY(hipMemsetAsync(cnt, 0, sizeof(int32_t), st));
        hipLaunchKernelGGL(k_pick, dim3(gr), dim3(64), 0, st, n_reads, sbeg, send, d_seeds, d_read_off, d_read_len,
                           order, chain_of, cwin, d_ext, d_out, av, nav, pos, p, cnt, jsi, jrun, joff, jlen, jseed,
                           jwin);
        CH_TRY(hipGetLastError());
        CH_TRY(hipMemcpyAsync(h, cnt, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        CH_TRY(hipStreamSynchronize(st));
        cs->check_ms += ms_since(tc);
        const int32_t nj = h[0];
        if (nj == 0) break;
        const auto te = std::chrono::steady_clock::now();
        const int rc = extend_seeds_device_win(ctx, opt, d_reads, joff, jlen, jseed, jwin, nj, jout, nullptr);
        if (rc) return rc;
        cs->ext_ms += ms_since(te);
        bsw_ext_stats_t es{};
        get_ext_stats(ctx, &es);
        for (int q = 0; q < 4; ++q) cs->n_pairs[q] += es.n_pairs[q];
        cs->kernel_ms += es.kernel_ms;
        hipLaunchKernelGGL(k_scatter, dim3((unsigned)((nj + 255) / 256)), dim3(256), 0, st, nj, jsi, jrun, jout, sbeg,
                           d_out, d_ext, av, nav);
        CH_TRY(hipGetLastError());
        cs->rounds++;
        cs->n_extended += nj;
    }
    CH_TRY(hipStreamSynchronize(st));
    cs->n_skipped = ns - cs->n_extended;
    return BSW_OK;
}

}  // namespace bsw

extern "C" int bsw_chain2aln_device(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *d_reads,
                                    const int64_t *read_off, const int32_t *read_len, int32_t n_reads,
                                    const bsw_seed_t *seeds, const int32_t *seed_read, const int32_t *seed_chain,
                                    int32_t n_seeds, bsw_alnreg_t *out, int32_t *extended)
{
    if (!ctx || !opt || n_seeds < 0 || n_reads < 0 ||
        (n_seeds > 0 && (!d_reads || !read_off || !read_len || !seeds || !seed_read || !seed_chain || !out ||
                         !extended)))
        return BSW_E_INVAL;
    if (n_seeds == 0) {
        bsw::set_chain_stats(ctx, bsw_chain_stats_t{});
        return BSW_OK;
    }
    // host inputs up, the GPU rounds (bsw_chain.hip), regions down
    if (hipSetDevice(bsw::ctx_device(ctx)) != hipSuccess) return BSW_E_HIP;
    void *d[7] = {};
    const size_t sz[7] = {sizeof(int64_t) * (size_t)n_reads, sizeof(int32_t) * (size_t)n_reads,
                          sizeof(bsw_seed_t) * (size_t)n_seeds, sizeof(int32_t) * (size_t)n_seeds,
                          sizeof(int32_t) * (size_t)n_seeds, sizeof(bsw_alnreg_t) * (size_t)n_seeds,
                          sizeof(int32_t) * (size_t)n_seeds};
    int rc = BSW_OK;
    const int dev = bsw::ctx_device(ctx);
    for (int k = 0; k < 7 && rc == BSW_OK; ++k)
        if (bsw::devcache_get(dev, std::max<size_t>(sz[k], 1), &d[k]) != hipSuccess) rc = BSW_E_NOMEM;
    const void *src[5] = {read_off, read_len, seeds, seed_read, seed_chain};
    for (int k = 0; k < 5 && rc == BSW_OK; ++k)
        if (hipMemcpy(d[k], src[k], sz[k], hipMemcpyHostToDevice) != hipSuccess) rc = BSW_E_HIP;
    bsw_chain_stats_t cs{};
    if (rc == BSW_OK)
        rc = bsw::chain_rounds_device(ctx, opt, d_reads, (const int64_t *)d[0], (const int32_t *)d[1], n_reads,
                                      (const bsw_seed_t *)d[2], (const int32_t *)d[3], (const int32_t *)d[4], n_seeds,
                                      (bsw_alnreg_t *)d[5], (int32_t *)d[6], &cs);
    if (rc == BSW_OK && (hipMemcpy(out, d[5], sz[5], hipMemcpyDeviceToHost) != hipSuccess ||
                         hipMemcpy(extended, d[6], sz[6], hipMemcpyDeviceToHost) != hipSuccess))
        rc = BSW_E_HIP;
    // nothing is queued on these blocks here: the copies are blocking, chain_rounds_device drains
    // its lease stream on every path (LeaseGuard) and the extension calls it makes drain their
    // slots' streams, failed or not (DeviceCtx::give_back) -- so no device-wide synchronise, which
    // would stall every other caller's work on the GPU
    for (int k = 0; k < 7; ++k)
        bsw::devcache_put(dev, d[k], std::max<size_t>(sz[k], 1));
    bsw::set_chain_stats(ctx, cs);
    return rc;
}

extern "C" int bsw_chain2aln_resident(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *d_reads,
                                      const int64_t *d_read_off, const int32_t *d_read_len, int32_t n_reads,
                                      const bsw_seed_t *d_seeds, const int32_t *d_seed_read,
                                      const int32_t *d_seed_chain, int32_t n_seeds, bsw_alnreg_t *d_out,
                                      int32_t *d_extended)
{
    if (!ctx || !opt || n_seeds < 0 || n_reads < 0 ||
        (n_seeds > 0 && (!d_reads || !d_read_off || !d_read_len || !d_seeds || !d_seed_read || !d_seed_chain ||
                         !d_out || !d_extended)))
        return BSW_E_INVAL;
    bsw_chain_stats_t cs{};
    const int rc = bsw::chain_rounds_device(ctx, opt, d_reads, d_read_off, d_read_len, n_reads, d_seeds, d_seed_read,
                                            d_seed_chain, n_seeds, d_out, d_extended, &cs);
    bsw::set_chain_stats(ctx, cs);
    return rc;
}

