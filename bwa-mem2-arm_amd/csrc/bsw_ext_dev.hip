// bsw_ext_dev.hip -- the extension pipeline (include/bsw_ext.h) with
// every per-read step on the GPU: job building, band-retry selection and local / to-end
// interpretation are small one-thread-per-read kernels around the batch engine, against a
// reference kept RESIDENT in HBM (bsw_set_reference: a 3 Gb genome is ~1% of one MI355X's
// 288 GB), so a call moves only reads + seeds in and regions out.  Semantics are exactly those
// of the host builder bsw_ext.cpp (and of the CPU oracle oracle/ext_ref.c): see bsw_ext.h.
//
// Layout: jobs are SPARSE -- job slot i belongs to read i (an empty SeqPair, len 0, when read i
// has no extension on that side), so no compaction is needed; the engine's plan / sort puts
// the empty slots in their own cheap wavefronts.  Code buffers use fixed per-read strides
// (qstride = the longest seeded read, tstride = the longest target window either side uses,
// both found by ext_scan): LEFT writes the reversed query prefix and the reversed window, RIGHT
// the forward suffix and window.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "bsw_ext_k.h"
#include "bsw_wave.h"

namespace bsw {

__device__ __forceinline__ int cal_max_gap_d(const ExtDevParams &p, int qlen)
{
    const int l_del = (int)((double)(qlen * p.a - p.o_del) / p.e_del + 1.);
    const int l_ins = (int)((double)(qlen * p.a - p.o_ins) / p.e_ins + 1.);
    int l = max(l_del, l_ins);
    l = max(l, 1);
    return min(l, p.w << 1);
}

// mem_chain2aln's target window of one seed taken as a chain of one (bsw_ext.cpp chain_window)
__device__ __forceinline__ void seed_window_d(const ExtDevParams &p, const bsw_seed_t &s, int l, int64_t *r0,
                                              int64_t *r1)
{
    const int qe = s.qbeg + s.len;
    int64_t lo = s.rbeg - (s.qbeg + cal_max_gap_d(p, s.qbeg));
    int64_t hi = s.rbeg + s.len + ((l - qe) + cal_max_gap_d(p, l - qe));
    lo = lo > 0 ? lo : 0;
    hi = hi < p.ref_len ? hi : p.ref_len;
    if (p.l_pac > 0 && lo < p.l_pac && p.l_pac < hi) {
        if (s.rbeg < p.l_pac) hi = p.l_pac;
        else lo = p.l_pac;
    }
    *r0 = lo;
    *r1 = hi;
}

// Per read: validation and the target window (given per job in win, else the seed's own) into
// wout; per block (LDS), then one global atomic per block and word into slot blockIdx % 32 (own
// 64-B line): meta[slot * 16 + k], k = 0 max read length, 1 input error, 2 / 3 LEFT / RIGHT job
// counts, 4 longest target window.  A seeded read is rejected exactly as the host form rejects
// it (bsw_ext.cpp): seed outside the read / reference or across l_pac, read or either side's
// window longer than BSW_MAX_LEN, a given window that does not hold the seed.
__global__ void ext_scan_kernel(const ExtDevParams p, const int32_t *__restrict__ read_len,
                                const bsw_seed_t *__restrict__ seeds, const int64_t *__restrict__ win, int32_t n,
                                int64_t *__restrict__ wout, int32_t *__restrict__ meta)
{
    __shared__ int s_m[5];
    if (threadIdx.x < 5) s_m[threadIdx.x] = 0;
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int l = 0, err = 0, nl = 0, nr = 0, tl = 0;
    if (i < n) {
        const bsw_seed_t s = seeds[i];
        int64_t r0 = 0, r1 = 0;
        if (s.len > 0) {            // only seeded reads are validated and sized (as bsw_extend_seeds)
            l = read_len[i];
            if (l < 0 || l > BSW_MAX_LEN || s.qbeg < 0 || s.qbeg + s.len > l || s.rbeg < 0 ||
                s.rbeg + s.len > p.ref_len || (p.l_pac > 0 && s.rbeg < p.l_pac && s.rbeg + s.len > p.l_pac)) {
                err = 1;
            } else {
                if (win) {
                    r0 = win[2 * i];
                    r1 = win[2 * i + 1];
                } else {
                    seed_window_d(p, s, l, &r0, &r1);
                }
                const int64_t lt = s.rbeg - r0, rt = r1 - (s.rbeg + s.len);
                if (lt < 0 || rt < 0 || lt > BSW_MAX_LEN || rt > BSW_MAX_LEN) {
                    err = 1;
                } else {
                    nl = s.qbeg > 0;
                    nr = s.qbeg + s.len < l;
                    tl = (int)max(nl ? lt : 0, nr ? rt : 0);
                }
            }
            if (err) l = 0;
        }
        wout[2 * i] = r0;
        wout[2 * i + 1] = r1;
    }
    const int lane = threadIdx.x & 63;
    const int wl = wave_max(l), wt = wave_max(tl);
    const unsigned long long be = __ballot(err), bl = __ballot(nl), br = __ballot(nr);
    if (lane == 0) {
        atomicMax(&s_m[0], wl);
        if (be) atomicOr(&s_m[1], 1);
        if (bl) atomicAdd(&s_m[2], __popcll(bl));
        if (br) atomicAdd(&s_m[3], __popcll(br));
        atomicMax(&s_m[4], wt);
    }
    __syncthreads();
    int32_t *slot = meta + (blockIdx.x % kExtMetaSpread) * 16;
    if (threadIdx.x == 0 && s_m[0]) atomicMax(&slot[0], s_m[0]);
    if (threadIdx.x == 1 && s_m[1]) atomicOr(&slot[1], 1);
    if (threadIdx.x == 2 && s_m[2]) atomicAdd(&slot[2], s_m[2]);
    if (threadIdx.x == 3 && s_m[3]) atomicAdd(&slot[3], s_m[3]);
    if (threadIdx.x == 4 && s_m[4]) atomicMax(&slot[4], s_m[4]);
}

__global__ void ext_left_build_kernel(const ExtDevParams p, const uint8_t *__restrict__ reads,
                                      const int64_t *__restrict__ read_off, const int32_t *__restrict__ read_len,
                                      const bsw_seed_t *__restrict__ seeds, const int64_t *__restrict__ win,
                                      int32_t n, const uint8_t *__restrict__ ref, ExtState *__restrict__ st,
                                      SeqPair *__restrict__ pairs, uint8_t *__restrict__ qbuf,
                                      uint8_t *__restrict__ tbuf, bsw_alnreg_t *__restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    bsw_alnreg_t r;
    r.rb = r.re = 0; r.qb = r.qe = r.score = r.truesc = r.w = r.seedlen0 = 0;
    ExtState x;
    x.rmax0 = x.rmax1 = 0; x.score = x.prev = 0; x.lw = x.rw = p.w;
    SeqPair sp{};
    sp.id = i;
    const bsw_seed_t s = seeds[i];
    if (s.len > 0) {
        const int l = read_len[i];
        x.rmax0 = win[2 * i];                           // the window ext_scan validated
        x.rmax1 = win[2 * i + 1];
        r.seedlen0 = s.len;
        r.score = r.truesc = s.len * p.a;               // no-extension defaults (mem_chain2aln)
        r.qb = 0; r.rb = s.rbeg;
        r.qe = l; r.re = s.rbeg + s.len;
        x.score = s.len * p.a;
        if (s.qbeg > 0) {                               // reversed prefix / reversed window (ext_copy)
            const int tlen = (int)(s.rbeg - x.rmax0);
            sp.idr = i * p.tstride; sp.idq = i * p.qstride;
            sp.len1 = tlen; sp.len2 = s.qbeg; sp.h0 = s.len * p.a;
        }
    }
    out[i] = r;
    st[i] = x;
    pairs[i] = sp;
}

__global__ void ext_right_build_kernel(const ExtDevParams p, const uint8_t *__restrict__ reads,
                                       const int64_t *__restrict__ read_off, const int32_t *__restrict__ read_len,
                                       const bsw_seed_t *__restrict__ seeds, int32_t n, const uint8_t *__restrict__ ref,
                                       ExtState *__restrict__ st, SeqPair *__restrict__ pairs,
                                       uint8_t *__restrict__ qbuf, uint8_t *__restrict__ tbuf)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SeqPair sp{};
    sp.id = i;
    const bsw_seed_t s = seeds[i];
    const int l = read_len[i], qe = s.qbeg + s.len;
    if (s.len > 0 && qe < l) {                          // forward suffix / forward window (ext_copy)
        ExtState &x = st[i];
        const int64_t t0 = s.rbeg + s.len;
        const int tlen = (int)(x.rmax1 - t0);
        sp.idr = i * p.tstride; sp.idq = i * p.qstride;
        sp.len1 = tlen; sp.len2 = l - qe; sp.h0 = x.score;
        x.prev = x.score;                               // a->score before the band loop
    }
    pairs[i] = sp;
}

// Code-buffer fill for the jobs the build kernel laid out: 16 lanes per job, so each byte
// load / store instruction covers 16 consecutive bytes of 4 jobs (the one-thread-per-read form
// touched 64 cache lines per instruction).  LEFT: reversed prefix / window ending at rbeg;
// RIGHT: forward suffix / window from rbeg + len.
__global__ void ext_copy_kernel(int left, const uint8_t *__restrict__ reads, const int64_t *__restrict__ read_off,
                                const bsw_seed_t *__restrict__ seeds, int32_t n, const uint8_t *__restrict__ ref,
                                const SeqPair *__restrict__ pairs, uint8_t *__restrict__ qbuf,
                                uint8_t *__restrict__ tbuf)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int i = (int)(t >> 4), sub = (int)(t & 15);
    if (i >= n) return;
    const SeqPair sp = pairs[i];
    if (sp.len2 <= 0) return;
    const bsw_seed_t s = seeds[i];
    const uint8_t *q = reads + read_off[i];
    uint8_t *qd = qbuf + sp.idq, *td = tbuf + sp.idr;
    if (left) {
        for (int k = sub; k < sp.len2; k += 16) qd[k] = q[s.qbeg - 1 - k];
        for (int k = sub; k < sp.len1; k += 16) td[k] = ref[s.rbeg - 1 - k];
    } else {
        const int qe = s.qbeg + s.len;
        const int64_t t0 = s.rbeg + s.len;
        for (int k = sub; k < sp.len2; k += 16) qd[k] = q[qe + k];
        for (int k = sub; k < sp.len1; k += 16) td[k] = ref[t0 + k];
    }
}

// Band retry t: a job of src (pairs for t == 1, the previous retry batch after) is redone with
// w << t when its score changed and max_off >= 3/4 of the band it ran with (wt); sub[i] gets
// the job or an empty slot.
__global__ void ext_retry_mark_kernel(const SeqPair *__restrict__ src, SeqPair *__restrict__ sub,
                                      ExtState *__restrict__ st, int32_t n, int32_t wt, int32_t *__restrict__ cnt)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SeqPair p = src[i];
    const bool redo = p.len2 > 0 && !(p.score == st[i].prev || p.max_off < (wt >> 1) + (wt >> 2));
    if (redo) {
        st[i].prev = p.score;
        atomicAdd(cnt, 1);
    } else {
        p = SeqPair{};
        p.id = i;
    }
    sub[i] = p;
}

__global__ void ext_retry_merge_kernel(SeqPair *__restrict__ pairs, const SeqPair *__restrict__ sub,
                                       ExtState *__restrict__ st, int32_t n, int32_t wn, int left)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (sub[i].len2 > 0) {
        pairs[i] = sub[i];
        if (left) st[i].lw = wn;
        else st[i].rw = wn;
    }
}

// local vs to-end (mem_chain2aln): LEFT with pen_clip5, RIGHT with pen_clip3
__global__ void ext_interp_kernel(const ExtDevParams p, const int32_t *__restrict__ read_len,
                                  const bsw_seed_t *__restrict__ seeds, int32_t n, const SeqPair *__restrict__ pairs,
                                  ExtState *__restrict__ st, bsw_alnreg_t *__restrict__ out, int left)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SeqPair sp = pairs[i];
    if (sp.len2 <= 0) {
        if (!left && seeds[i].len > 0) out[i].w = max(st[i].lw, st[i].rw);
        return;
    }
    const bsw_seed_t s = seeds[i];
    bsw_alnreg_t r = out[i];
    ExtState &x = st[i];
    if (left) {
        r.score = sp.score;
        if (sp.gscore <= 0 || sp.gscore <= sp.score - p.pen_clip5) {
            r.qb = s.qbeg - sp.qle; r.rb = s.rbeg - sp.tle; r.truesc = sp.score;
        } else {
            r.qb = 0; r.rb = s.rbeg - sp.gtle; r.truesc = sp.gscore;
        }
    } else {
        const int sc0 = x.score, qe = s.qbeg + s.len;
        r.score = sp.score;
        if (sp.gscore <= 0 || sp.gscore <= sp.score - p.pen_clip3) {
            r.qe = qe + sp.qle; r.re = s.rbeg + s.len + sp.tle; r.truesc += sp.score - sc0;
        } else {
            r.qe = read_len[i]; r.re = s.rbeg + s.len + sp.gtle; r.truesc += sp.gscore - sc0;
        }
        r.w = max(x.lw, x.rw);
    }
    x.score = sp.score;
    out[i] = r;
}

static inline dim3 grid_of(int32_t n) { return dim3((unsigned)((n + 255) / 256)); }

hipError_t launch_ext_scan(const ExtDevParams &p, const int32_t *read_len, const bsw_seed_t *seeds, const int64_t *win,
                           int32_t n, int64_t *wout, int32_t *meta, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(meta, 0, kExtMetaSpread * 16 * sizeof(int32_t), s);
    if (e != hipSuccess || n <= 0) return e;
    hipLaunchKernelGGL(ext_scan_kernel, grid_of(n), dim3(256), 0, s, p, read_len, seeds, win, n, wout, meta);
    return hipGetLastError();
}

hipError_t launch_ext_build(int left, const ExtDevParams &p, const uint8_t *reads, const int64_t *read_off,
                            const int32_t *read_len, const bsw_seed_t *seeds, const int64_t *win, int32_t n,
                            const uint8_t *ref, ExtState *st, SeqPair *pairs, uint8_t *qbuf, uint8_t *tbuf,
                            bsw_alnreg_t *out, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    if (left)
        hipLaunchKernelGGL(ext_left_build_kernel, grid_of(n), dim3(256), 0, s, p, reads, read_off, read_len, seeds,
                           win, n, ref, st, pairs, qbuf, tbuf, out);
    else
        hipLaunchKernelGGL(ext_right_build_kernel, grid_of(n), dim3(256), 0, s, p, reads, read_off, read_len, seeds,
                           n, ref, st, pairs, qbuf, tbuf);
    hipLaunchKernelGGL(ext_copy_kernel, dim3((unsigned)(((int64_t)n * 16 + 255) / 256)), dim3(256), 0, s, left, reads,
                       read_off, seeds, n, ref, pairs, qbuf, tbuf);
    return hipGetLastError();
}

hipError_t launch_ext_retry_mark(const SeqPair *src, SeqPair *sub, ExtState *st, int32_t n, int32_t wt,
                                 int32_t *cnt, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(cnt, 0, sizeof(int32_t), s);
    if (e != hipSuccess || n <= 0) return e;
    hipLaunchKernelGGL(ext_retry_mark_kernel, grid_of(n), dim3(256), 0, s, src, sub, st, n, wt, cnt);
    return hipGetLastError();
}

hipError_t launch_ext_retry_merge(SeqPair *pairs, const SeqPair *sub, ExtState *st, int32_t n, int32_t wn,
                                  int left, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ext_retry_merge_kernel, grid_of(n), dim3(256), 0, s, pairs, sub, st, n, wn, left);
    return hipGetLastError();
}

hipError_t launch_ext_interp(int left, const ExtDevParams &p, const int32_t *read_len, const bsw_seed_t *seeds,
                             int32_t n, const SeqPair *pairs, ExtState *st, bsw_alnreg_t *out, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ext_interp_kernel, grid_of(n), dim3(256), 0, s, p, read_len, seeds, n, pairs, st, out, left);
    return hipGetLastError();
}

}  // namespace bsw
