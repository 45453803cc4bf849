// bsw_host.cpp -- host engine behind the C ABI (include/bsw.h).
//
// Replaces upstream BandedPairWiseSW's batch wrapper (smithWatermanBatchWrapper16/8:
// sort -> pad -> AoS->SoA -> kernel -> write back; SURVEY.md §3.2,
// docs-archive/WEEK1_WRAPPER_COMPLETE.md:27-118) with an MI355X pipeline that keeps the
// upstream AoS layout in HBM and does the "transpose" implicitly (one lane per pair):
//
//   plan_kernel   : per pair -> kernel class (lane QMAX bucket 32..160 | wide) + sort key
//                   (class, qlen desc, tlen desc) so every wavefront gets 64 like-shaped pairs
//   radix sort    : hipCUB DeviceRadixSort on the 27-bit key -> order[] (= sortPairsLen)
//   DP kernels    : one launch per non-empty class over its slice of order[]
//   results       : written by the kernels straight into the SeqPair records
//
// Concurrency: upstream calls getScores* from kt_for workers; every call here takes a Slot
// (own HIP stream + device buffers) from a per-device pool, so calls are reentrant.
// Host-buffer calls on an n_gpus context shard the batch by contiguous pair ranges across
// devices (one host thread per device) -- pairs are independent.
// Errors are returned as BSW_E* codes; there is no CPU path in this library.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <type_traits>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <deque>
#include <condition_variable>
#include <vector>
#include "../../include/bsw.h"
#include "bsw_kernels.h"
#include "bsw_mate_k.h"
#include "bsw_global_k.h"
#include "bsw_ext_k.h"
#include <chrono>
#include "bsw_internal.h"
#include "bsw_pool.h"
#include <emmintrin.h>

namespace bsw {

constexpr int kNumLaneClasses = 5;          // QMAX 32, 64, 96, 128, 160
constexpr int kPkClass0 = kNumLaneClasses;  // packed kernel, same QMAX buckets (classes 5..9)
constexpr int kWideClass = kPkClass0 + kNumLaneClasses;   // index of the wide-kernel class
constexpr int kWvClass0 = kWideClass + 1;   // wave-per-alignment kernel, 4 / 8 / 16 columns per lane
constexpr int kNumWvClasses = 3;
constexpr int kWvCols[kNumWvClasses] = {4, 8, 16};
constexpr int kNumClasses = kWvClass0 + kNumWvClasses;
constexpr int kMetaCounts = 16;             // class counters per slot (one 64-B line per slot)
constexpr int kMetaSpread = 32;             // slots: block b adds into slot b % 32 (no hot line)
constexpr int kMetaMaxq = kMetaCounts * kMetaSpread;   // d_meta: counts[32][16], maxq_wide, err
constexpr int kMetaErr = kMetaMaxq + 1;
constexpr int kMetaFlag = kMetaErr + 1;     // row-group kernel: a pair outside its contract
constexpr int kMetaCnt = kMetaFlag + 1;     // extension pipeline: band-retry count readback
constexpr int kMetaWords = kMetaCnt + 1;
constexpr int kKeyBits = 32;                // 4 class + 8 qlen + 1 related + 11 tlen + 8 h0 bits
static_assert(kNumClasses <= kMetaCounts, "class counts");

// Lifetime predictor for the sort key (scheduling only, results never depend on it): does the
// query look like an extension of the target near the seed?  Identity of query[10, 40) with
// target[10 + s, 40 + s), best over |s| <= 6; > 18 of 30 matches = related.  Unrelated pairs
// die within a few dozen rows and shrink their band ends on the way; giving them their own
// wavefronts keeps the related waves' band edges uniform (masked groups
// 25% -> 11% at C2 in simulation).  The identity count itself is the next sort field: it tracks
// the pair's score along the first rows, hence its band-end trajectory and its lifetime.
__device__ __forceinline__ int seed_matches(const uint8_t *__restrict__ q, int qlen,
                                            const uint8_t *__restrict__ r, int tlen)
{
    if (qlen < 40 || tlen < 46) return 31;
    uint8_t qb[30], rb[42];
#pragma unroll
    for (int j = 0; j < 30; ++j) qb[j] = q[10 + j];
#pragma unroll
    for (int j = 0; j < 42; ++j) rb[j] = r[4 + j];
    int best = 0;
#pragma unroll
    for (int sft = 0; sft <= 12; ++sft) {
        int c = 0;
#pragma unroll
        for (int j = 0; j < 30; ++j) c += qb[j] == rb[j + sft];
        best = max(best, c);
    }
    return best;                    // identities of the best shift (of 30); > 18: related
}

// Per pair: class + sort key.  Lane classes need qlen <= QMAX and int16-safe scores.
// Wave-kernel class for a pair (bsw_wv.hip contract), -1 if it does not qualify.
__device__ __forceinline__ int wv_class(const KParams &kp, int32_t w, int qlen, int tlen, int h0)
{
    if (kp.maxsc != 1 || qlen > kWvQmax || h0 < 0) return -1;
    if ((int64_t)kp.e_ins * qlen >= 2700) return -1;
    // E and F live in int16 lanes updated by wrapping v_pk_sub_i16 (bsw_wv.hip): keep the gap
    // steps far from the int16 range
    if (128 + kp.o_del + 2 * kp.e_del >= 30000 || 128 + kp.o_ins + 2 * kp.e_ins >= 30000) return -1;
    if ((int64_t)h0 + min(qlen, tlen) + (int64_t)kp.e_ins * (qlen + 1) >= 30000) return -1;
    int wl = w;
    const int ni = qlen * kp.maxsc + kp.end_bonus - kp.o_ins;
    const int nd = qlen * kp.maxsc + kp.end_bonus - kp.o_del;
    wl = min(wl, max((ni + kp.e_ins) / kp.e_ins, 1));
    wl = min(wl, max((nd + kp.e_del) / kp.e_del, 1));
    for (int k = 0; k < kNumWvClasses; ++k)
        if (2 * wl + kWvCols[k] + 2 <= 64 * kWvCols[k]) return kWvClass0 + k;
    return -1;
}

__global__ void plan_kernel(const SeqPair *__restrict__ pairs, int32_t n, const KParams kp, int32_t w,
                            int32_t pc_route, int32_t wv_route, const uint8_t *__restrict__ ref,
                            const uint8_t *__restrict__ qer, uint32_t *__restrict__ keys,
                            int32_t *__restrict__ vals, int32_t *__restrict__ counts,
                            int32_t *__restrict__ maxq_wide, int keymode, int misroute)
{
    const int maxsc = kp.maxsc;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < n;
    SeqPair p{};
    if (valid) p = pairs[i];
    const int qlen = max(p.len2, 0), tlen = max(p.len1, 0);
    const int64_t hi = (int64_t)max(p.h0, 0) + (int64_t)max(maxsc, 0) * min(qlen, tlen);
    int c = kWideClass;
    // queries past the register kernels' 160 columns: the wave-per-alignment kernel
    // (BSW_OPT_LONG 1, default); BSW_OPT_LONG 2 sends every qualifying pair there (tests)
    const int wvc = wv_route ? wv_class(kp, w, qlen, tlen, p.h0) : -1;
    if (wv_route == 2 && wvc >= 0) c = wvc;
    else if (hi < 32768 && p.h0 >= 0) {
        if (qlen <= 32) c = 0;
        else if (qlen <= 64) c = 1;
        else if (qlen <= 96) c = 2;
        else if (qlen <= 128) c = 3;
        else if (qlen <= 160) c = 4;
        // 8-bit score regime (key H << 8 | j fits 16 bits, H <= h0 + min(qlen, tlen)) -> the
        // packed-column kernel (needs qlen < QMAX: bucket by qlen + 1)
        if (pc_route && c < kNumLaneClasses && p.h0 + min(qlen, tlen) <= 255 && qlen + 1 <= 160)
            c = kPkClass0 + (qlen + 1 <= 32 ? 0 : qlen + 1 <= 64 ? 1 : qlen + 1 <= 96 ? 2 : qlen + 1 <= 128 ? 3 : 4);
    }
    if (c == kWideClass && wvc >= 0) c = wvc;
    if (misroute) c = 0;          // BSW_OPT_TEST_MISROUTE: the QMAX=32 lane kernel's guard must trip
    if (valid) {
        if (c == kWideClass) atomicMax(maxq_wide, qlen);
        // (class, qlen desc, related first, tlen desc, h0 desc): like-shaped pairs share a
        // wavefront; equal h0 and relatedness give lanes similar band-end trajectories
        const int mt = (c == kWideClass) ? 31 : seed_matches(qer + p.idq, qlen, ref + p.idr, tlen);
        const int rel = mt > 18;
        // sort key (scheduling only; results never depend on it).  Default: (class, qlen desc,
        // related first, tlen / 32 desc, seed identities desc, h0 desc) -- pairs that align
        // alike share a wavefront, so their band ends move together (C2 kernel 9.58 -> 8.60 ms vs
        // the h0-only order, BSW_SORTKEY=0)
        if (keymode == 0)
            keys[i] = ((uint32_t)c << 28) | ((uint32_t)(255 - min(qlen, 255)) << 20) |
                      ((uint32_t)(1 - rel) << 19) | ((uint32_t)(2047 - min(tlen, 2047)) << 8) |
                      (uint32_t)(255 - min(max(p.h0, 0), 255));
        else
            keys[i] = ((uint32_t)c << 28) | ((uint32_t)(255 - min(qlen, 255)) << 20) |
                      ((uint32_t)(1 - rel) << 19) | ((uint32_t)(63 - min(tlen >> 5, 63)) << 13) |
                      ((uint32_t)(31 - min(mt, 31)) << 8) | (uint32_t)(255 - min(max(p.h0, 0), 255));
        vals[i] = i;
    }
    // class counts: wave ballots -> LDS per block -> one global add per block and class into the
    // block's slot (32 slots in separate 64-B lines; same-line atomics from every wave cost
    // ~10 ns each, 0.16-0.7 ms per 1M pairs)
    __shared__ int s_cnt[kNumClasses];
    if (threadIdx.x < kNumClasses) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kNumClasses; ++k) {
        const unsigned long long m = __ballot(valid && c == k);
        if (m && lane == __ffsll((long long)m) - 1) atomicAdd(&s_cnt[k], __popcll(m));
    }
    __syncthreads();
    if (threadIdx.x < kNumClasses && s_cnt[threadIdx.x])
        atomicAdd(&counts[(blockIdx.x % kMetaSpread) * kMetaCounts + threadIdx.x], s_cnt[threadIdx.x]);
}

// one device call: run_plan's arguments, kept in the slot for run_dp
struct PlanCall {
    SeqPair *d_pairs = nullptr;
    const uint8_t *d_ref = nullptr, *d_qer = nullptr;
    int32_t n = 0, w = 0;
    int cell_bits = 16;
    hipStream_t stream = nullptr;
    hipStream_t dp_stream = nullptr;    // the DP kernels' stream when not `stream` (host pipeline:
                                        //   everything else of a chunk runs on the helper stream)
    hipStream_t plan_stream = nullptr;  // plan + sort stream when not the slot's pstream
    // row-group kernel contract as the host checked it: gq_maxq >= 0 = every pair fits (longest
    // query gq_maxq, longest target gq_maxt); -2 = not checked (the kernel flags misfits, run_dp
    // falls back to the planned path); -1 = some pair does not fit (planned path at once)
    int gq_maxq = -2, gq_maxt = 0;
    int32_t *d_out24 = nullptr;         // row-group kernel, host-checked batch: outputs as 6 x int32
                                        //   per pair here instead of into d_pairs
};

struct Slot {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // device buffers (grown on demand)
    SeqPair *d_pairs = nullptr; size_t cap_pairs = 0;
    uint8_t *d_ref = nullptr; size_t cap_ref = 0;
    uint8_t *d_qer = nullptr; size_t cap_qer = 0;
    uint32_t *d_keys = nullptr, *d_keys2 = nullptr;
    int32_t *d_vals = nullptr, *d_order = nullptr; size_t cap_sort = 0;
    void *d_tmp = nullptr; size_t cap_tmp = 0;
    int32_t *d_meta = nullptr;          // counts[kMetaCounts], maxq_wide, err
    int32_t *h_meta = nullptr;          // pinned mirror
    int2 *d_scratch = nullptr; size_t cap_scratch = 0;
    // host-buffer pipeline: pinned staging of one chunk and its device copy
    void *h_stage = nullptr; size_t cap_stage = 0;
    uint8_t *d_stage = nullptr; size_t cap_dstage = 0;
    int32_t *d_bkt = nullptr; size_t cap_bkt = 0;   // staged exceptions: first word per 4096 positions
    // mate rescue (bsw_mate.h)
    int32_t *d_mjobs = nullptr; size_t cap_mjobs = 0;
    uint16_t *d_mrows = nullptr; size_t cap_mrows = 0;
    int32_t *d_mmeta = nullptr, *h_mmeta = nullptr;
    unsigned long long *d_mcells = nullptr;
    SeqPair *d_mpairs = nullptr; size_t cap_mpairs = 0;
    bsw_kswr_t *d_maln = nullptr; size_t cap_maln = 0;
    hipEvent_t ev2 = nullptr, ev3 = nullptr;
    // global alignment (bsw_global.h)
    uint32_t *d_gz = nullptr; size_t cap_gz = 0;
    int32_t *d_gmeta = nullptr, *h_gmeta = nullptr;
    uint32_t *d_gcig = nullptr; size_t cap_gcig = 0;
    int32_t *d_gncig = nullptr; size_t cap_gncig = 0;
    int32_t *d_gretry = nullptr; size_t cap_gretry = 0;   // narrow-window traceback retries: count, list
    // device extension pipeline (bsw_ext_dev.hip)
    SeqPair *d_xpairs = nullptr, *d_xsub = nullptr; size_t cap_xpairs = 0, cap_xsub = 0;
    uint8_t *d_xq = nullptr, *d_xt = nullptr; size_t cap_xq = 0, cap_xt = 0;
    ExtState *d_xst = nullptr; size_t cap_xst = 0;
    int64_t *d_xwin = nullptr; size_t cap_xwin = 0;   // per-read target windows (ext_scan)
    // class launches of one batch fork over side streams (independent pairs; small batches are
    // bound by the longest wave of each class, so classes run side by side instead of in turn)
    static constexpr int kSide = 3;
    hipStream_t side[kSide] = {};
    hipEvent_t evf = nullptr, evj[kSide] = {};
    bool timed = false;
    hipStream_t run_stream = nullptr;   // stream of the last run_device (finish_stats waits on it)
    bsw_stats_t stats{};
    hipEvent_t evm = nullptr;           // class-count readback of the last run_plan
    hipStream_t pstream = nullptr;      // high-priority stream of run_plan
    hipEvent_t evh = nullptr;           // inputs ready on the call's stream (pstream waits)
    hipEvent_t evd = nullptr;           // host pipeline: a chunk's DP done (its outputs' readback waits)
    PlanCall plan;                      // arguments of the last run_plan (run_dp's input)
    bool ownq = false;                  // `stream` has a hardware queue of its own (DeviceCtx::acquire)
    int fast = 0;                       // last run_plan launched the row-group kernel: 2 = host-
                                        //   checked batch, 1 = kernel-checked (flag read back)
};

static int hip_rc(hipError_t e)
{
    if (e == hipSuccess) return BSW_OK;
    if (e == hipErrorOutOfMemory) return BSW_E_NOMEM;
    return BSW_E_HIP;
}
#define BSW_TRY(x) do { hipError_t _e = (x); if (_e != hipSuccess) return ::bsw::hip_rc(_e); } while (0)

// BSW_OPT_TEST_FAIL_ALLOC: this many upcoming buffer growths fail as out of memory (tests of the
// host-buffer call's recovery, bsw.h); process-wide, 0 in production
static std::atomic<int> g_fail_alloc{0};
static bool inject_nomem()
{
    int v = g_fail_alloc.load(std::memory_order_relaxed);
    while (v > 0)
        if (g_fail_alloc.compare_exchange_weak(v, v - 1)) return true;
    return false;
}

template <class T>
static hipError_t grow(T *&p, size_t &cap, size_t need)   // cap counts elements (bytes for void)
{
    if (need <= cap) return hipSuccess;
    if (inject_nomem()) return hipErrorOutOfMemory;
    // 25% headroom: the pipeline's chunks vary (ramp, a merged remainder up to 1.25x) and slots
    // rotate between them, so exact-fit growth reallocated on many calls (hipFree syncs the device)
    const size_t n = std::max(need + need / 4, cap * 3 / 2);
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    constexpr size_t esz = std::is_void<T>::value ? 1 : sizeof(typename std::conditional<std::is_void<T>::value, char, T>::type);
    hipError_t e = hipMalloc((void **)&p, n * esz);
    if (e == hipSuccess) cap = n;
    return e;
}

struct AggReq;
struct DeviceCtx {
    int device = 0;
    std::atomic<int> inflight{0};       // host-buffer calls running on this logical device
    // cross-call coalescing (coalesced_call): small host-buffer calls queue here; up to
    // agg_leaders_max of their threads at a time each run everything queued as ONE batch
    std::mutex agg_mu;
    std::condition_variable agg_cv;
    std::deque<AggReq *> agg_q;
    int64_t agg_qn = 0;                 // pairs queued in agg_q
    int64_t agg_run = 0;                // pairs in the batches on the device
    int agg_nrun = 0;                   // batches on the device
    int agg_inside = 0;                 // callers inside coalesced_call
    int agg_lingering = 0;              // leaders waiting for a deeper queue
    int agg_leaders = 0;
    int agg_leaders_max = 4;            // BSW_OPT_COALESCE_LEADERS
    int agg_linger_us = 20;             // BSW_OPT_COALESCE_LINGER (20 us since round 6: 8 callers x 1K
                                        //   +15-30%, 16 equal or better, <= 4 never linger)
    std::atomic<int> ownq_n{0};         // slots whose stream got a hardware queue of its own (acquire)
    std::atomic<bool> copies_warm{false};   // host_shard's copy-engine warm-up ran (prime_copies)
    std::mutex mu;
    std::vector<std::unique_ptr<Slot>> free_slots;
    uint8_t *d_refres = nullptr;        // resident reference (bsw_set_reference)
    int64_t refres_len = -1;
    std::shared_mutex refmu;            // extension calls hold it shared while they use d_refres

    ~DeviceCtx()
    {
        for (auto &s : free_slots) release_slot(s.get());
        if (d_refres) { (void)hipSetDevice(device); (void)hipFree(d_refres); }
    }
    void release_slot(Slot *s)
    {
        if (s->ownq) ownq_n.fetch_sub(1);
        (void)hipSetDevice(s->device);
        (void)hipFree(s->d_pairs); (void)hipFree(s->d_ref); (void)hipFree(s->d_qer);
        (void)hipFree(s->d_keys); (void)hipFree(s->d_keys2); (void)hipFree(s->d_vals); (void)hipFree(s->d_order);
        (void)hipFree(s->d_tmp); (void)hipFree(s->d_meta); (void)hipFree(s->d_scratch);
        (void)hipFree(s->d_stage);
        (void)hipFree(s->d_bkt);
        if (s->h_stage) (void)hipHostFree(s->h_stage);
        (void)hipFree(s->d_mjobs); (void)hipFree(s->d_mrows); (void)hipFree(s->d_mmeta);
        (void)hipFree(s->d_mcells); (void)hipFree(s->d_mpairs); (void)hipFree(s->d_maln);
        if (s->h_mmeta) (void)hipHostFree(s->h_mmeta);
        (void)hipFree(s->d_gz); (void)hipFree(s->d_gmeta); (void)hipFree(s->d_gcig); (void)hipFree(s->d_gncig);
        (void)hipFree(s->d_gretry);
        if (s->h_gmeta) (void)hipHostFree(s->h_gmeta);
        (void)hipFree(s->d_xpairs); (void)hipFree(s->d_xsub); (void)hipFree(s->d_xq); (void)hipFree(s->d_xt);
        (void)hipFree(s->d_xst);
        (void)hipFree(s->d_xwin);
        if (s->ev2) (void)hipEventDestroy(s->ev2);
        if (s->ev3) (void)hipEventDestroy(s->ev3);
        if (s->h_meta) (void)hipHostFree(s->h_meta);
        if (s->ev0) (void)hipEventDestroy(s->ev0);
        if (s->evm) (void)hipEventDestroy(s->evm);
        if (s->evh) (void)hipEventDestroy(s->evh);
        if (s->evd) (void)hipEventDestroy(s->evd);
        if (s->pstream) (void)hipStreamDestroy(s->pstream);
        if (s->ev1) (void)hipEventDestroy(s->ev1);
        if (s->stream) (void)hipStreamDestroy(s->stream);
        for (int k = 0; k < Slot::kSide; ++k) {
            if (s->side[k]) (void)hipStreamDestroy(s->side[k]);
            if (s->evj[k]) (void)hipEventDestroy(s->evj[k]);
        }
        if (s->evf) (void)hipEventDestroy(s->evf);
    }
    std::unique_ptr<Slot> acquire(int &rc)
    {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!free_slots.empty()) {
                auto s = std::move(free_slots.back());
                free_slots.pop_back();
                rc = BSW_OK;
                return s;
            }
        }
        auto s = std::make_unique<Slot>();
        s->device = device;
        rc = hip_rc(hipSetDevice(device));
        if (rc) return nullptr;
        // The slot's stream through a CU mask of EVERY CU: a masked stream gets a hardware queue of its
        // own, so concurrent kt_for-sized calls do not share the runtime's four queues
        // (GPU_MAX_HW_QUEUES) and serialise their kernels behind each other.  Measured (percall_bench,
        // 8 C++ callers, same box x2, profiles/r05/slot_ownq_percall.txt): 1K pairs per call without
        // coalescing 9.4-9.5 -> 10.7-11.0 M/s, 4K 30.4-30.8 -> 34.7-34.9, 10K 40.5-40.9 -> 42.1-42.5;
        // 1M-pair host calls unchanged.  The first 16 slots of a device.
        // A CU-masked stream is a BLOCKING stream (hipExtStreamCreateWithCUMask takes no flags): it
        // orders against the legacy null stream.  The library itself issues nothing on the null
        // stream (its copies run on non-blocking streams of its own: bsw_set_reference, the FM-index
        // build); a caller's own null-stream work waits for, and is waited on by, these slots'
        // kernels ("Streams")
        bool made = false;
        if (ownq_n.fetch_add(1) < 16) {
            hipDeviceProp_t pr;
            if (hipGetDeviceProperties(&pr, device) == hipSuccess && pr.multiProcessorCount > 0 &&
                pr.multiProcessorCount <= 1024) {
                uint32_t m[32] = {};
                const int ncu = pr.multiProcessorCount;
                for (int c = 0; c < ncu; ++c) m[c / 32] |= 1u << (c % 32);
                made = hipExtStreamCreateWithCUMask(&s->stream, (uint32_t)((ncu + 31) / 32), m) == hipSuccess;
            }
            s->ownq = made;
            if (!made) ownq_n.fetch_sub(1);
        } else {
            ownq_n.fetch_sub(1);
        }
        if (!made && (rc = hip_rc(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)))) return nullptr;
        if ((rc = hip_rc(hipEventCreate(&s->ev0)))) return nullptr;
        if ((rc = hip_rc(hipEventCreate(&s->ev1)))) return nullptr;
        if ((rc = hip_rc(hipMalloc((void **)&s->d_meta, kMetaWords * sizeof(int32_t))))) return nullptr;
        if ((rc = hip_rc(hipHostMalloc((void **)&s->h_meta, kMetaWords * sizeof(int32_t), 0)))) return nullptr;
        return s;
    }
    // free every cached slot (streams, events, device and pinned buffers): the first step of a
    // failed call's recovery (scores_eb), so its rerun allocates afresh.  Slots other calls hold
    // are untouched; they come back to the pool as usual
    void trim()
    {
        std::vector<std::unique_ptr<Slot>> v;
        {
            std::lock_guard<std::mutex> g(mu);
            v.swap(free_slots);
        }
        for (auto &s : v) release_slot(s.get());
    }
    // rc != 0: the call failed part-way and may have left work queued on the slot's streams
    // (or the caller's stream it ran on) that still reads or writes the slot's buffers -- drain
    // it before another call can take the slot
    void give_back(std::unique_ptr<Slot> s, int rc = 0)
    {
        if (rc) {
            (void)hipSetDevice(s->device);
            for (hipStream_t st : {s->stream, s->pstream, s->run_stream, s->side[0], s->side[1],
                                   s->side[2]})
                if (st) (void)hipStreamSynchronize(st);
        }
        std::lock_guard<std::mutex> g(mu);
        free_slots.push_back(std::move(s));
    }
};

}  // namespace bsw

struct bsw_ctx {
    bsw_params_t params;
    bsw::KParams kp;
    std::vector<std::unique_ptr<bsw::DeviceCtx>> devs;
    std::mutex stats_mu;
    bsw_stats_t last{};
    bsw_ext_stats_t ext_last{};
    bsw_chain_stats_t chain_last{};
    bsw_mate_stats_t mate_last{};
    bsw_global_stats_t glob_last{};
    struct Pinned { std::mutex mu; void *p = nullptr; size_t cap = 0; } pin[2];
    int glob_band = 0;                  // BSW_OPT_GLOB_BAND
    int64_t ext_chunk = 0;              // BSW_OPT_EXT_CHUNK (0: the int32-offset bound)
    int32_t host_chunk = 196608;        // BSW_OPT_HOST_CHUNK: pairs per host-buffer pipeline chunk (round 6:
                                        //   48 blocks beat 64 by 3-4% per 1M-pair call on two boxes,
                                        //   profiles/r06/host_chunk_sweep.txt)
    int host_pack = 2;                  // BSW_OPT_HOST_PACK: 2-bit (2) or nibble (4) staging
    int64_t split_min = 131072;         // BSW_OPT_SPLIT_MIN: smaller calls go whole to one device
    int32_t coalesce = 8192;            // BSW_OPT_COALESCE: calls of <= this many pairs coalesce
    std::atomic<unsigned> rr{0};        // tie-break rotation of the one-device pick
    ~bsw_ctx()
    {
        for (auto &b : pin)
            if (b.p) (void)hipHostFree(b.p);
    }
};

namespace bsw {

static void make_kparams(const bsw_params_t &p, KParams &kp)
{
    memset(&kp, 0, sizeof(kp));
    kp.o_del = p.o_del; kp.e_del = p.e_del; kp.o_ins = p.o_ins; kp.e_ins = p.e_ins;
    kp.zdrop = p.zdrop; kp.end_bonus = p.end_bonus;
    int mx = 0;
    for (int i = 0; i < 25; ++i) mx = std::max(mx, (int)p.mat[i]);
    kp.maxsc = mx;
    memcpy(kp.mat, p.mat, 25);
    // prof[t] byte q = mat[t][q] for q < 5; q = 5..7 (invalid codes) score as N
    for (int t = 0; t < 8; ++t) {
        const int tt = std::min(t, 4);
        uint8_t b[8];
        for (int q = 0; q < 8; ++q) b[q] = (uint8_t)p.mat[tt * 5 + std::min(q, 4)];
        kp.prof[t][0] = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
        kp.prof[t][1] = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
    }
    // packed-column kernel scoring contract (bsw_pc.hip): match 1, one mismatch value in
    // [-127, -1], every N entry -1, symmetric gap penalties.
    bool ok = p.o_del == p.o_ins && p.e_del == p.e_ins && p.e_del > 0 && p.o_del + p.e_del < 4096;
    const int mis = p.mat[1];
    ok = ok && mis < 0 && mis >= -127;
    for (int a = 0; a < 5 && ok; ++a)
        for (int b = 0; b < 5 && ok; ++b) {
            const int v = p.mat[a * 5 + b];
            ok = (a == 4 || b == 4) ? v == -1 : (a == b ? v == 1 : v == mis);
        }
    kp.pk_ok = ok ? 1 : 0;
    // routing / scheduling defaults; bsw_set_option changes them per context
    kp.kern8 = 1;
    kp.keymode = 2;
    kp.misroute = 0;
    kp.fork = 1;
    kp.long_route = 1;
    kp.small_batch = 32768;          // 16-lane row-group form up to 32K pairs
    kp.mid_batch = 32768;
    kp.group_kernel = 1;
    // the row-group kernel's 32-lane latency form for batches of at most 2048 pairs: 1K calls 0.277
    // -> 0.25 ms, 8 callers without coalescing +8%; from 4K pairs the 16-lane form's fewer
    // instructions per cell win (percall_bench, same box, profiles/r05/gq32_percall.txt)
    kp.gq32_max = 2048;
}

// keys / keys2 / vals / order (radix-sort buffers) grow together
static hipError_t grow_sort(Slot &s, int32_t n)
{
    if ((size_t)n <= s.cap_sort) return hipSuccess;
    (void)hipFree(s.d_keys); (void)hipFree(s.d_keys2); (void)hipFree(s.d_vals); (void)hipFree(s.d_order);
    s.d_keys = s.d_keys2 = nullptr; s.d_vals = s.d_order = nullptr; s.cap_sort = 0;
    const size_t cap = std::max((size_t)n, (size_t)1024);
    hipError_t e;
    if ((e = hipMalloc((void **)&s.d_keys, cap * sizeof(uint32_t))) != hipSuccess) return e;
    if ((e = hipMalloc((void **)&s.d_keys2, cap * sizeof(uint32_t))) != hipSuccess) return e;
    if ((e = hipMalloc((void **)&s.d_vals, cap * sizeof(int32_t))) != hipSuccess) return e;
    if ((e = hipMalloc((void **)&s.d_order, cap * sizeof(int32_t))) != hipSuccess) return e;
    s.cap_sort = cap;
    return hipSuccess;
}

// The device pipeline on one slot's device; d_* are device pointers valid on `stream`, in two
// halves so a host pipeline can stage the next chunk between them:
//   run_plan : enqueue plan -> sort -> the class-count readback (nothing waits)
//   run_dp   : wait for that readback, enqueue the DP kernels and the readback of their
//              range-guard word into h_meta[kMetaErr]
// finish_stats() waits for the rest and turns a tripped guard into BSW_E_RANGE.
// the slot's high-priority stream (created on first use)
static int ensure_pstream(Slot &s)
{
    if (!s.pstream) {
        int lo = 0, hi = 0;
        BSW_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        BSW_TRY(hipStreamCreateWithPriority(&s.pstream, hipStreamNonBlocking, hi));
        BSW_TRY(hipEventCreateWithFlags(&s.evh, hipEventDisableTiming));
    }
    return BSW_OK;
}

static int run_plan(const KParams &kp, Slot &s, const PlanCall &pc)
{
    s.stats = bsw_stats_t{};
    s.timed = false;
    s.run_stream = pc.stream;
    s.plan = pc;
    s.fast = 0;
    if (pc.n == 0) return BSW_OK;
    const int32_t n = pc.n;
    // small batches (kt_for-sized calls): the row-group kernel (bsw_gq.hip) straight on the
    // call's stream -- no plan, no sort, no class-count readback
    // medium batches: the quad form (4 lanes per pair, targets <= 512 bytes); at most
    // kp.gq32_max pairs: the 32-lane latency form (two DPP rows per pair, ~21% fewer instructions
    // per row; BSW_OPT_GQ32_MAX) -- within the small-batch range (BSW_OPT_SMALL_BATCH 0 keeps every
    // batch off the 16/32-lane forms)
    const int32_t gq32_max = std::min<int32_t>(kp.gq32_max, kp.small_batch);
    const int gs = n <= gq32_max ? 32 : n <= kp.small_batch ? 16 : 4;
    const bool gq_size = n <= kp.small_batch || n <= kp.mid_batch;
    const bool gq_fit = pc.gq_maxq == -2 || (pc.gq_maxq >= 0 && (gs >= 16 || pc.gq_maxt <= 512));
    if (kp.group_kernel && gq_size && gq_fit && kp.long_route == 1 && kp.maxsc == 1 && !kp.misroute) {
        const bool checked = pc.gq_maxq >= 0;
        const int cols = checked ? gq_cols_for(pc.gq_maxq, gs) : (gs == 32 ? 6 : gs == 16 ? 10 : 40);
        int32_t *d_err = s.d_meta + kMetaErr;
        // the DP stream when the call has one (host pipeline: the helper stream holds few CUs)
        hipStream_t fs = pc.stream;
        if (pc.dp_stream && pc.dp_stream != pc.stream) {
            if (int r = ensure_pstream(s)) return r;           // (creates evh)
            BSW_TRY(hipEventRecord(s.evh, pc.stream));
            BSW_TRY(hipStreamWaitEvent(pc.dp_stream, s.evh, 0));
            fs = pc.dp_stream;
            s.run_stream = fs;
        }
        if (!pc.d_out24)                       // (the staged path's input kernel zeroed them)
            BSW_TRY(hipMemsetAsync(d_err, 0, 2 * sizeof(int32_t), fs));
        BSW_TRY(hipEventRecord(s.ev0, fs));
        BSW_TRY(launch_gq_kernel(gs, cols, kp, pc.w, pc.d_pairs, nullptr, n, pc.d_ref, pc.d_qer,
                                 d_err, checked ? nullptr : s.d_meta + kMetaFlag, checked ? pc.d_out24 : nullptr,
                                 fs));
        BSW_TRY(hipEventRecord(s.ev1, fs));
        BSW_TRY(hipMemcpyAsync(s.h_meta + kMetaErr, d_err, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, fs));
        if (!checked) {
            if (!s.evm) BSW_TRY(hipEventCreateWithFlags(&s.evm, hipEventDisableTiming));
            BSW_TRY(hipEventRecord(s.evm, fs));
        }
        s.stats.n_launches = 1;
        s.stats.n_i16 = n;
        s.stats.n_group = n;
        s.fast = checked ? 2 : 1;
        return BSW_OK;
    }
    // plan + sort run on the slot's high-priority stream (ordered after the call's stream by an
    // event): while other chunks' DP kernels fill the GPU, their few blocks are dispatched
    // first instead of queuing behind thousands of DP workgroups (it delays the next chunk's
    // DP launch otherwise: 1-3 ms per chunk in the host pipeline's trace)
    if (int r = ensure_pstream(s)) return r;
    hipStream_t stream = pc.plan_stream ? pc.plan_stream : s.pstream;
    if (pc.stream != stream) {
        BSW_TRY(hipEventRecord(s.evh, pc.stream));
        BSW_TRY(hipStreamWaitEvent(stream, s.evh, 0));
    }
    BSW_TRY(grow_sort(s, n));
    BSW_TRY(hipMemsetAsync(s.d_meta, 0, kMetaWords * sizeof(int32_t), stream));
    int32_t *d_counts = s.d_meta, *d_maxq = s.d_meta + kMetaMaxq;
    // pairs in the 8-bit score regime (h0 + min(qlen, tlen) <= 255, bwa-style scoring) take the
    // packed-column kernel on both entry points (getScores8 / getScores16: identical results,
    // fewer instructions per cell), the rest the int16 lane kernel (on cell_bits = 8: the
    // overflow fallback) or the int32 wide kernel
    const int pc_route = (kp.pk_ok && kp.kern8) ? 1 : 0;
    // small batches (upstream's kt_for workers hand over a few thousand pairs per call): one
    // lane-per-pair wave lives ~1.2 ms whatever the batch size, so they are latency-bound; the
    // wave-per-alignment kernel spreads each pair over 64 lanes -- 0.35 vs 1.39 ms per call at
    // 1K C2 pairs, 1.05 vs 1.58 at 10K, slower past ~20K
    const int32_t long_route = (kp.long_route == 1 && n <= kp.small_batch) ? 2 : kp.long_route;
    hipLaunchKernelGGL(plan_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                       pc.d_pairs, n, kp, pc.w, pc_route, long_route, pc.d_ref, pc.d_qer, s.d_keys,
                       s.d_vals, d_counts, d_maxq, (int)kp.keymode, (int)kp.misroute);
    BSW_TRY(hipGetLastError());
    size_t tmp_bytes = 0;
    BSW_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, s.d_keys, s.d_keys2, s.d_vals,
                                               s.d_order, n, 0, kKeyBits, stream));
    BSW_TRY(grow(s.d_tmp, s.cap_tmp, tmp_bytes));
    BSW_TRY(hipcub::DeviceRadixSort::SortPairs(s.d_tmp, tmp_bytes, s.d_keys, s.d_keys2, s.d_vals,
                                               s.d_order, n, 0, kKeyBits, stream));
    BSW_TRY(hipMemcpyAsync(s.h_meta, s.d_meta, kMetaWords * sizeof(int32_t), hipMemcpyDeviceToHost, stream));
    if (!s.evm) BSW_TRY(hipEventCreateWithFlags(&s.evm, hipEventDisableTiming));
    BSW_TRY(hipEventRecord(s.evm, stream));
    return BSW_OK;
}

static int run_dp(const KParams &kp, Slot &s)
{
    const PlanCall &pc = s.plan;
    if (pc.n == 0) return BSW_OK;
    hipStream_t stream = pc.dp_stream && !s.fast ? pc.dp_stream : pc.stream;
    const int32_t w = pc.w;
    const int cell_bits = pc.cell_bits;
    SeqPair *d_pairs = pc.d_pairs;
    const uint8_t *d_ref = pc.d_ref, *d_qer = pc.d_qer;
    int32_t *d_err = s.d_meta + kMetaErr;
    if (s.fast) {
        if (s.fast == 1) {
            BSW_TRY(hipEventSynchronize(s.evm));   // the row-group kernel's misfit flag
            if (s.h_meta[kMetaFlag] != 0) {
                // some pair is outside the row-group kernel's contract: the whole batch again on
                // the planned path (identical outputs; rare -- long or int16-unsafe pairs)
                PlanCall again = pc;
                again.gq_maxq = -1;
                const int r = run_plan(kp, s, again);
                if (r) return r;
                return run_dp(kp, s);
            }
        }
        s.timed = true;                            // ev0 / ev1 bracket the kernel; the guard
        return BSW_OK;                             //   word is on its way to h_meta[kMetaErr]
    }
    BSW_TRY(hipEventSynchronize(s.evm));           // the class counts are in h_meta
    BSW_TRY(hipStreamWaitEvent(stream, s.evm, 0)); // order / meta written on the plan stream
    int32_t counts[kNumClasses] = {};
    for (int sl = 0; sl < kMetaSpread; ++sl)
        for (int c = 0; c < kNumClasses; ++c) counts[c] += s.h_meta[sl * kMetaCounts + c];
    const int32_t maxq_wide = s.h_meta[kMetaMaxq];
    // DP kernels, one launch per non-empty class; event-timed as the hot region.  With more than
    // one class the launches fork over the slot's side streams and join back on `stream`.
    int nclass = 0;
    for (int c = 0; c < kNumClasses; ++c) nclass += counts[c] > 0;
    const bool fork = nclass > 1 && kp.fork;
    BSW_TRY(hipEventRecord(s.ev0, stream));
    if (fork) {
        if (!s.evf) BSW_TRY(hipEventCreateWithFlags(&s.evf, hipEventDisableTiming));
        for (int k = 0; k < Slot::kSide; ++k)
            if (!s.side[k]) {
                BSW_TRY(hipStreamCreateWithFlags(&s.side[k], hipStreamNonBlocking));
                BSW_TRY(hipEventCreateWithFlags(&s.evj[k], hipEventDisableTiming));
            }
        BSW_TRY(hipEventRecord(s.evf, stream));
        for (int k = 0; k < Slot::kSide; ++k) BSW_TRY(hipStreamWaitEvent(s.side[k], s.evf, 0));
    }
    int nl = 0;                        // launch k runs on stream k mod (1 + kSide)
    auto next_stream = [&]() {
        const int k = nl++ % (1 + Slot::kSide);
        return (fork && k > 0) ? s.side[k - 1] : stream;
    };
    // every launch of the fork; the join below runs whatever happens here, so no side stream
    // can still be reading this slot's buffers when the slot goes back to the pool
    const int lrc = [&]() -> int {
        int32_t off = 0;
        for (int c = 0; c < kNumLaneClasses; ++c) {
            if (counts[c] > 0) {
                BSW_TRY(launch_lane_kernel(kLaneQmax[c], kp, w, d_pairs, s.d_order + off, counts[c],
                                           d_ref, d_qer, d_err, next_stream()));
                s.stats.n_launches++;
                s.stats.n_i16 += counts[c];
            }
            off += counts[c];
        }
        for (int c = 0; c < kNumLaneClasses; ++c) {
            const int32_t np = counts[kPkClass0 + c];
            if (np > 0) {
                BSW_TRY(launch_pc_kernel(kLaneQmax[c], kp, w, d_pairs, s.d_order + off, np, d_ref, d_qer,
                                         d_err, next_stream()));
                s.stats.n_launches++;
                s.stats.n_packed += np;
                if (cell_bits == 8) s.stats.n_u8 += np;
                else s.stats.n_i16 += np;
            }
            off += np;
        }
        if (counts[kWideClass] > 0) {
            const int32_t nw = counts[kWideClass];
            const size_t need = (size_t)(maxq_wide + 2) * (size_t)nw;
            BSW_TRY(grow(s.d_scratch, s.cap_scratch, need));
            BSW_TRY(launch_wide_kernel(kp, w, d_pairs, s.d_order + off, nw, d_ref, d_qer, s.d_scratch,
                                       nw, next_stream()));
            s.stats.n_launches++;
            s.stats.n_wide += nw;
        }
        off += counts[kWideClass];
        for (int c = 0; c < kNumWvClasses; ++c) {
            const int32_t nv = counts[kWvClass0 + c];
            if (nv > 0) {
                BSW_TRY(launch_wv_kernel(kWvCols[c], kp, w, d_pairs, s.d_order + off, nv, d_ref, d_qer, d_err,
                                         next_stream()));
                s.stats.n_launches++;
                s.stats.n_i16 += nv;
                s.stats.n_wave += nv;
            }
            off += nv;
        }
        return BSW_OK;
    }();
    if (fork)
        for (int k = 0; k < Slot::kSide; ++k) {
            BSW_TRY(hipEventRecord(s.evj[k], s.side[k]));
            BSW_TRY(hipStreamWaitEvent(stream, s.evj[k], 0));
        }
    if (lrc) {
        (void)hipStreamSynchronize(stream);         // drain what was queued before the failure
        return lrc;
    }
    BSW_TRY(hipEventRecord(s.ev1, stream));
    // the DP kernels' range guard (a pair routed to a class that cannot hold it) -> host,
    // after every DP launch of this batch
    BSW_TRY(hipMemcpyAsync(s.h_meta + kMetaErr, d_err, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
    s.run_stream = stream;
    s.timed = true;
    return BSW_OK;
}

static int run_device(const KParams &kp, Slot &s, SeqPair *d_pairs, const uint8_t *d_ref,
                      const uint8_t *d_qer, int32_t n, int32_t w, int cell_bits, hipStream_t stream)
{
    PlanCall pc;
    pc.d_pairs = d_pairs; pc.d_ref = d_ref; pc.d_qer = d_qer;
    pc.n = n; pc.w = w; pc.cell_bits = cell_bits; pc.stream = stream;
    int r = run_plan(kp, s, pc);
    if (r) return r;
    return run_dp(kp, s);
}

// Wait for run_device's work (through the guard readback), record the DP kernel time; a
// tripped range guard is BSW_E_RANGE (the affected pairs' outputs were not written).
static int finish_stats(Slot &s, bool spin = false)
{
    if (s.timed) {
        float ms = 0.f;
        s.timed = false;
        if (spin) {         // a short batch: poll instead of the runtime's blocking wait (wake-up latency)
            hipError_t q;
            while ((q = hipStreamQuery(s.run_stream)) == hipErrorNotReady) _mm_pause();
            BSW_TRY(q);
        }
        BSW_TRY(hipStreamSynchronize(s.run_stream));
        BSW_TRY(hipEventElapsedTime(&ms, s.ev0, s.ev1));
        s.stats.kernel_ms = ms;
        if (s.h_meta[kMetaErr] != 0) return BSW_E_RANGE;
    }
    return BSW_OK;
}

static void par_pack_nibbles(uint8_t *dst, const uint8_t *src, size_t nbytes)
{
    constexpr size_t kPiece = (size_t)2 << 20;
    const int nt = (int)std::min<size_t>(HostPool::workers() + 1, nbytes / kPiece);
    if (nt <= 1) { pack_nibbles(dst, src, nbytes); return; }
    auto cut = [=](size_t t) { return t == (size_t)nt ? nbytes : (nbytes * t / nt) & ~(size_t)31; };
    HostPool::get().parallel_for(nt, [=](int t) {
        const size_t a = cut(t), b = cut(t + 1);
        pack_nibbles(dst + a / 2, src + a, b - a);
    });
}

// bytes out[0, n) from nibbles in[0, (n + 1) / 2): 4 packed bytes -> 8 codes per thread
__global__ void unpack_kernel(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int64_t n)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t o = t * 8;
    if (o >= n) return;
    uint32_t v = 0;
    const int64_t ib = t * 4, nin = (n + 1) / 2;
    if (ib + 4 <= nin) v = *(const uint32_t *)(in + ib);
    else
        for (int k = 0; k < 4 && ib + k < nin; ++k) v |= (uint32_t)in[ib + k] << (8 * k);
    const uint32_t lo = (v & 0x0f0f0f0fu), hi = (v >> 4) & 0x0f0f0f0fu;
    // interleave: byte 2k = lo byte k, byte 2k + 1 = hi byte k
    const uint32_t w0 = __builtin_amdgcn_perm(hi, lo, 0x05010400u);
    const uint32_t w1 = __builtin_amdgcn_perm(hi, lo, 0x07030602u);
    if (o + 8 <= n) {
        *(uint2 *)(out + o) = make_uint2(w0, w1);
    } else {
        const uint8_t b[8] = {(uint8_t)w0, (uint8_t)(w0 >> 8), (uint8_t)(w0 >> 16), (uint8_t)(w0 >> 24),
                              (uint8_t)w1, (uint8_t)(w1 >> 8), (uint8_t)(w1 >> 16), (uint8_t)(w1 >> 24)};
        for (int k = 0; o + k < n; ++k) out[o + k] = b[k];
    }
}

// bytes out[0, n) from 2-bit codes in[0, (n + 3) / 4): 4 packed bytes -> 16 codes per thread
__global__ void unpack2_kernel(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int64_t n)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t o = t * 16;
    if (o >= n) return;
    uint32_t v = 0;
    const int64_t ib = t * 4, nin = (n + 3) / 4;
    if (ib + 4 <= nin) v = *(const uint32_t *)(in + ib);
    else
        for (int k = 0; k < 4 && ib + k < nin; ++k) v |= (uint32_t)in[ib + k] << (8 * k);
    // plane p holds code 4m + p in byte m; output dword m = byte m of planes 0..3
    const uint32_t p0 = v & 0x03030303u, p1 = (v >> 2) & 0x03030303u;
    const uint32_t p2 = (v >> 4) & 0x03030303u, p3 = (v >> 6) & 0x03030303u;
    const uint32_t a01 = __builtin_amdgcn_perm(p1, p0, 0x05010400u), b01 = __builtin_amdgcn_perm(p1, p0, 0x07030602u);
    const uint32_t a23 = __builtin_amdgcn_perm(p3, p2, 0x05010400u), b23 = __builtin_amdgcn_perm(p3, p2, 0x07030602u);
    const uint4 r = make_uint4(__builtin_amdgcn_perm(a23, a01, 0x05040100u), __builtin_amdgcn_perm(a23, a01, 0x07060302u),
                               __builtin_amdgcn_perm(b23, b01, 0x05040100u), __builtin_amdgcn_perm(b23, b01, 0x07060302u));
    if (o + 16 <= n) {
        *(uint4 *)(out + o) = r;
    } else {
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
        for (int k = 0; o + k < n; ++k) out[o + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
}

// (PairIn: the kernels' input fields of a SeqPair, bsw_kernels.h)

__global__ void expand_pairs_kernel(const PairIn *__restrict__ in, SeqPair *__restrict__ out, int32_t n)
{
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const PairIn p = in[i];
    SeqPair sp;
    memset(&sp, 0, sizeof(sp));
    sp.idr = p.idr; sp.idq = p.idq; sp.len1 = p.len1; sp.len2 = p.len2; sp.h0 = p.h0;
    out[i] = sp;
}

// The whole staged input of a coalesced batch in one launch (what unpack2 x2 + patch_codes +
// expand_pairs + two pad memsets did in six): index space = ref 16-code units, qer units, pairs.
// Exception words (pos << 2 | code bits 2-3, bsw_pack.cpp) are ascending per buffer.  A lane
// unpacks 64 codes (16 packed bytes in, 64 bytes out; see unpack_unit for the interleaving), a wave 4096 consecutive positions: the
// wave reads the index of its first exception from exc_bucket_kernel's table (one entry per 4096
// positions), loads the next 64 words (one per lane) and every lane patches the ones inside its
// own codes from a uniform walk over those in the wave's range (~4 per wave at bwa's N rate).  A
// binary search per lane per 16 codes -- ~20 dependent loads each at 900K exceptions per 3M-pair
// piece -- made the staging kernel latency-bound: 1.8-3.0 ms per 3M pairs in the RCCL leg's trace,
// ahead of every piece's DP; one search per wave still 1.2-2.4 ms (profiles/r06/rccl_leg_trace.txt).
// Whole-wave function: every lane of the wave calls it (valid = the lane has codes to write).
constexpr int kUnitCodes = 64;          // codes per lane
__device__ __forceinline__ uint4 unpack16(uint32_t v)    // 16 codes from 4 packed bytes
{
    const uint32_t p0 = v & 0x03030303u, p1 = (v >> 2) & 0x03030303u;
    const uint32_t p2 = (v >> 4) & 0x03030303u, p3 = (v >> 6) & 0x03030303u;
    const uint32_t a01 = __builtin_amdgcn_perm(p1, p0, 0x05010400u), b01 = __builtin_amdgcn_perm(p1, p0, 0x07030602u);
    const uint32_t a23 = __builtin_amdgcn_perm(p3, p2, 0x05010400u), b23 = __builtin_amdgcn_perm(p3, p2, 0x07030602u);
    return make_uint4(__builtin_amdgcn_perm(a23, a01, 0x05040100u), __builtin_amdgcn_perm(a23, a01, 0x07060302u),
                      __builtin_amdgcn_perm(b23, b01, 0x05040100u), __builtin_amdgcn_perm(b23, b01, 0x07060302u));
}
__device__ __forceinline__ void unpack_unit(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int64_t n,
                                            int64_t wave_t0, int64_t units,
                                            const uint32_t *__restrict__ exc, int32_t ne,
                                            const int32_t *__restrict__ bkt)
{
    // the wave's 4096 positions [W, W + 4096) as 4 sub-units per lane, interleaved so that every
    // load / store instruction of the wave is contiguous: sub-unit u of lane L = the 16 codes at
    // W + 1024 u + 16 L (4 packed bytes in, one 16-B store out)
    if (wave_t0 >= units) return;                                // (the tail waves of a block: uniform)
    const int lane = (int)(threadIdx.x & 63);
    const int64_t W = wave_t0 * kUnitCodes, nin = (n + 3) / 4;
    uint4 w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t pos = W + 1024 * u + 16 * lane, ib = pos / 4;
        uint32_t v = 0;
        if (ib + 4 <= nin) v = *(const uint32_t *)(in + ib);
        else
            for (int k = 0; k < 4 && ib + k < nin; ++k) v |= (uint32_t)in[ib + k] << (8 * k);
        w[u] = unpack16(v);
    }
    if (ne > 0) {
        const int64_t whi = W + 64 * kUnitCodes;
        const int32_t lo = min(max(bkt[wave_t0 / 64], 0), ne);  // first exception at or past W (uniform)
        for (int32_t base = lo;; base += 64) {                   // uniform: 64 words per round
            const int32_t j = base + lane;
            const uint32_t e = j < ne ? exc[j] : 0u;
            const bool in_w = j < ne && (int64_t)(e >> 2) < whi;
            const int cnt = __popcll(__ballot(in_w));              // sorted: lanes 0 .. cnt - 1
            for (int q = 0; q < cnt; ++q) {
                const uint32_t eq = (uint32_t)__shfl((int)e, q);
                const int64_t k = (int64_t)(eq >> 2) - W;         // 0 .. 4095 (in the wave's range)
                if (k >= 0 && k < 4096 && (int)((k >> 4) & 63) == lane) {
                    const int u = (int)(k >> 10), c = (int)(k & 15);
                    const uint32_t bits = (eq & 3u) << (8 * (c & 3) + 2);   // code bits 2-3
                    const int d = c >> 2;
#pragma unroll
                    for (int uu = 0; uu < 4; ++uu) {
                        w[uu].x |= (u == uu && d == 0) ? bits : 0u;
                        w[uu].y |= (u == uu && d == 1) ? bits : 0u;
                        w[uu].z |= (u == uu && d == 2) ? bits : 0u;
                        w[uu].w |= (u == uu && d == 3) ? bits : 0u;
                    }
                }
            }
            if (cnt < 64) break;
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t pos = W + 1024 * u + 16 * lane;
        if (pos + 16 <= n) {
            *(uint4 *)(out + pos) = w[u];
        } else {
            const uint32_t word[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
            for (int k = 0; pos + k < n; ++k) out[pos + k] = (uint8_t)(word[k >> 2] >> (8 * (k & 3)));
        }
    }
}

// Blocks of 256 threads, each block inside one segment (so every wave is): [ref 64-code units |
// qer units | records]; stage_in_grid() is the matching grid size
__host__ __device__ inline int64_t stage_in_blocks(int64_t r_tot, int64_t q_tot, int64_t n, int64_t *br, int64_t *bq)
{
    *br = ((r_tot + kUnitCodes - 1) / kUnitCodes + 255) / 256;
    *bq = ((q_tot + kUnitCodes - 1) / kUnitCodes + 255) / 256;
    return *br + *bq + (n + 255) / 256;
}

// bkt[b] = the first exception word at or past position 4096 b: ref buckets [0, nbr), then qer
// buckets [nbr, nbr + nbq) indexing the qer words (exc + n_r).  One lane per bucket, its own binary
// search: ~nbr + nbq lanes instead of one search per staging wave
__global__ void exc_bucket_kernel(const uint32_t *__restrict__ exc, int32_t n_r, int32_t ne, int64_t nbr, int64_t nbq,
                                  int32_t *__restrict__ bkt)
{
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nbr + nbq) return;
    const bool q = b >= nbr;
    const uint32_t *e = q ? exc + n_r : exc;
    const int64_t pos = (q ? b - nbr : b) * 4096;
    int32_t lo = 0, hi = q ? ne - n_r : n_r;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if ((int64_t)(e[mid] >> 2) < pos) lo = mid + 1; else hi = mid;
    }
    bkt[b] = lo;
}

__global__ __launch_bounds__(256) void stage_in_kernel(const uint8_t *__restrict__ ref2, int64_t r_tot,
                                const uint8_t *__restrict__ qer2,
                                int64_t q_tot, const uint32_t *__restrict__ exc, int32_t n_r, int32_t ne,
                                const PairIn *__restrict__ pin, int32_t n, uint8_t *__restrict__ ref,
                                uint8_t *__restrict__ qer, SeqPair *__restrict__ pairs, int32_t *__restrict__ zero2,
                                const int32_t *__restrict__ bkt, int64_t nbr)
{
    const int64_t tr = (r_tot + kUnitCodes - 1) / kUnitCodes, tq = (q_tot + kUnitCodes - 1) / kUnitCodes;   // lanes
    int64_t br, bq;
    stage_in_blocks(r_tot, q_tot, n, &br, &bq);
    const int64_t blk = blockIdx.x;
    const int wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (blk == 0 && threadIdx.x == 0) {
        *(uint32_t *)(ref + r_tot) = 0u;          // 4 zero bytes past each buffer
        *(uint32_t *)(qer + q_tot) = 0u;
        if (zero2) { zero2[0] = 0; zero2[1] = 0; }
    }
    if (blk < br) {
        unpack_unit(ref2, ref, r_tot, blk * 256 + 64 * wv, tr, exc, n_r, bkt);
        return;
    }
    if (blk < br + bq) {
        unpack_unit(qer2, qer, q_tot, (blk - br) * 256 + 64 * wv, tq, exc + n_r, ne - n_r, bkt + nbr);
        return;
    }
    const int64_t t = (blk - br - bq) * 256 + threadIdx.x;
    if (t < n) {
        const PairIn p = pin[t];
        SeqPair sp;
        memset(&sp, 0, sizeof(sp));
        sp.idr = p.idr; sp.idq = p.idq; sp.len1 = p.len1; sp.len2 = p.len2; sp.h0 = p.h0;
        pairs[t] = sp;
    }
}

static size_t exc_buckets(int64_t r_tot, int64_t q_tot) { return (size_t)((r_tot + 4095) / 4096 + (q_tot + 4095) / 4096 + 2); }

// The whole staged input of one batch: the exceptions' bucket table (when there are exceptions),
// then stage_in_kernel -- on `st`, the slot's d_bkt grown to the table
static int launch_stage_in(Slot &s, hipStream_t st, const uint8_t *ref2, int64_t r_tot, const uint8_t *qer2,
                           int64_t q_tot, const uint32_t *exc, int32_t n_r, int32_t ne, const PairIn *pin, int32_t n,
                           uint8_t *ref, uint8_t *qer, SeqPair *pairs, int32_t *zero2)
{
    const int64_t nbr = (r_tot + 4095) / 4096 + 1, nbq = (q_tot + 4095) / 4096 + 1;
    if (ne > 0) {
        BSW_TRY(grow(s.d_bkt, s.cap_bkt, exc_buckets(r_tot, q_tot)));
        hipLaunchKernelGGL(exc_bucket_kernel, dim3((unsigned)((nbr + nbq + 255) / 256)), dim3(256), 0, st, exc, n_r,
                           ne, nbr, nbq, s.d_bkt);
        BSW_TRY(hipGetLastError());
    }
    int64_t br, bq;
    const unsigned grid = (unsigned)stage_in_blocks(r_tot, q_tot, n, &br, &bq);
    hipLaunchKernelGGL(stage_in_kernel, dim3(grid), dim3(256), 0, st, ref2, r_tot, qer2, q_tot, exc, n_r, ne, pin, n,
                       ref, qer, pairs, zero2, (const int32_t *)s.d_bkt, nbr);
    return hip_rc(hipGetLastError());
}

// the six outputs of each pair (SeqPair bytes 32..55) -> 24 B per pair for the D2H
__global__ void gather_outputs_kernel(const SeqPair *__restrict__ in, int32_t *__restrict__ out, int32_t n)
{
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SeqPair &p = in[i];
    int32_t *o = out + 6 * (int64_t)i;
    o[0] = p.score; o[1] = p.tle; o[2] = p.gtle; o[3] = p.qle; o[4] = p.gscore; o[5] = p.max_off;
}

// Pre-pass of a host-buffer call, one parallel sweep over the records: validation (the ABI's
// BSW_E_RANGE before any device work) and per-block extents of the byte buffers, from which
// chunks are cut and staged without another pass.
constexpr int32_t kStageBlk = 4096;           // pairs per block (a chunk is whole blocks)
struct BlkStat {
    int64_t r_lo, r_hi, q_lo, q_hi, r_sum, q_sum;
    bool bad;
};

// blocks [b0, b1) of bs (sized for every block of the n pairs); false if any pair there is invalid
static bool prepass_range(const SeqPair *pairs, int32_t n, std::vector<BlkStat> &bs, int32_t b0, int32_t b1)
{
    auto blk = [&](int32_t b) {
        BlkStat t{INT64_MAX, 0, INT64_MAX, 0, 0, 0, false};
        const int32_t e = std::min(n, (b + 1) * kStageBlk);
        for (int32_t i = b * kStageBlk; i < e; ++i) {
            const SeqPair &p = pairs[i];
            t.bad |= p.len1 < 0 || p.len2 < 0 || p.len1 > BSW_MAX_LEN || p.len2 > BSW_MAX_LEN || p.idr < 0 ||
                     p.idq < 0;
            if (p.len1 > 0) { t.r_lo = std::min<int64_t>(t.r_lo, p.idr); t.r_hi = std::max<int64_t>(t.r_hi, (int64_t)p.idr + p.len1); t.r_sum += p.len1; }
            if (p.len2 > 0) { t.q_lo = std::min<int64_t>(t.q_lo, p.idq); t.q_hi = std::max<int64_t>(t.q_hi, (int64_t)p.idq + p.len2); t.q_sum += p.len2; }
        }
        bs[b] = t;
    };
    const int32_t nb = b1 - b0;
    if (nb < 16) {
        for (int32_t b = b0; b < b1; ++b) blk(b);
    } else {
        const int nt = std::min(HostPool::workers() + 1, (int)nb);
        HostPool::get().parallel_for(nt, [&](int t) {
            for (int32_t b = b0 + (int32_t)((int64_t)nb * t / nt); b < b0 + (int32_t)((int64_t)nb * (t + 1) / nt); ++b)
                blk(b);
        });
    }
    for (int32_t b = b0; b < b1; ++b)
        if (bs[b].bad) return false;
    return true;
}

static bool prepass(const SeqPair *pairs, int32_t n, std::vector<BlkStat> &bs)
{
    const int32_t nb = (n + kStageBlk - 1) / kStageBlk;
    bs.assign((size_t)nb, BlkStat{});
    return prepass_range(pairs, n, bs, 0, nb);
}

// One chunk of a host-buffer call staged in a slot's pinned buffer: [SeqPair x n | ref | qer].
// Contiguous chunks (the upstream layout: each batch's windows concatenated in pair order) pack
// their byte extents into 2-bit codes + exception words, with the records cut to their five
// input fields (20 of 56 B) and only the 24 output bytes coming back -- or into nibbles with
// whole records when the chunk holds too many non-ACGT bytes; scattered ones are
// gathered pair by pair as bytes and the staged records' idr / idq rewritten (only outputs
// ever go back to the caller).
enum StageMode { kStageGather = 0, kStageNibble = 1, kStage2bit = 2 };
struct StagedChunk {
    int32_t n = 0;
    int mode = kStageGather;
    bool packed = false;                // bulk extents (nibble or 2-bit)
    size_t pair_off = 0, ref_off = 0, qer_off = 0, exc_off = 0, bytes = 0;
    int32_t n_exr = 0, n_exq = 0;       // 2-bit: exception words for ref / qer
    size_t rb = 0, qb = 0;              // ref / qer bytes after unpacking
    int64_t r_base = 0, q_base = 0;     // staged ref byte 0 = caller byte r_base (bulk mode)
};

// blocks [b0, b1) = pairs [a, a + n)
// 2-bit staging of a bulk chunk: [PairIn x n | ref codes | qer codes | exception words], sized
// for at least the 24 B per pair of outputs that come back through the same buffers.  Returns 1
// (nothing staged) when the exception words would pass 1/32 of the bytes.
static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
static int stage_2bit(Slot &s, const SeqPair *pairs, const uint8_t *ref, const uint8_t *qer, int32_t n,
                      StagedChunk &c)
{
    const size_t rs = (c.rb + 3) / 4, qs = (c.qb + 3) / 4;
    const size_t exc_cap = (c.rb + c.qb) / 32 + 1024;
    c.pair_off = 0;
    c.ref_off = align256((size_t)n * sizeof(PairIn));
    c.qer_off = align256(c.ref_off + rs + 4);          // +4: the unpack's dword loads
    c.exc_off = align256(c.qer_off + qs + 4);
    c.bytes = std::max(c.exc_off + exc_cap * 4, (size_t)n * 24);
    if (c.bytes > s.cap_stage) {
        const size_t cap = std::max(c.bytes + c.bytes / 4, s.cap_stage * 3 / 2);
        if (s.h_stage) (void)hipHostFree(s.h_stage);
        s.h_stage = nullptr; s.cap_stage = 0;
        BSW_TRY(hipHostMalloc(&s.h_stage, cap, 0));
        s.cap_stage = cap;
    }
    uint8_t *h = (uint8_t *)s.h_stage;
    PairIn *pin = (PairIn *)(h + c.pair_off);
    const int np = (int)std::max<size_t>(1, ((size_t)n * sizeof(SeqPair)) >> 21);
    const int nr = (int)std::max<size_t>(1, c.rb >> 22), nq = (int)std::max<size_t>(1, c.qb >> 22);
    auto even = [](size_t total, int k, int parts) {     // piece bounds: multiples of 64 codes
        return k == parts ? total : (total * (size_t)k / (size_t)parts) & ~(size_t)63;
    };
    std::vector<std::vector<uint32_t>> ex((size_t)(nr + nq));
    HostPool::get().parallel_for(np + nr + nq, [&](int t) {
        if (t < np) {
            const int32_t a0 = (int32_t)((int64_t)n * t / np), a1 = (int32_t)((int64_t)n * (t + 1) / np);
            for (int32_t i = a0; i < a1; ++i)
                pin[i] = PairIn{pairs[i].idr, pairs[i].idq, pairs[i].len1, pairs[i].len2, pairs[i].h0};
        } else if (t < np + nr) {
            const size_t a0 = even(c.rb, t - np, nr), a1 = even(c.rb, t - np + 1, nr);
            pack_2bit(h + c.ref_off + a0 / 4, ref + a0, a1 - a0, (uint32_t)a0, ex[(size_t)(t - np)]);
        } else {
            const size_t a0 = even(c.qb, t - np - nr, nq), a1 = even(c.qb, t - np - nr + 1, nq);
            pack_2bit(h + c.qer_off + a0 / 4, qer + a0, a1 - a0, (uint32_t)a0, ex[(size_t)(t - np)]);
        }
    });
    size_t tot = 0, tr = 0;
    for (size_t k = 0; k < ex.size(); ++k) {
        tot += ex[k].size();
        if (k < (size_t)nr) tr += ex[k].size();
    }
    if (tot > exc_cap) return 1;
    uint32_t *exw = (uint32_t *)(h + c.exc_off);
    for (size_t k = 0, o = 0; k < ex.size(); o += ex[k].size(), ++k)
        if (!ex[k].empty()) memcpy(exw + o, ex[k].data(), ex[k].size() * 4);
    c.n_exr = (int32_t)tr;
    c.n_exq = (int32_t)(tot - tr);
    c.mode = kStage2bit;
    c.bytes = std::max(c.exc_off + tot * 4, (size_t)n * 24);
    memset(h + c.ref_off + rs, 0, 4);
    memset(h + c.qer_off + qs, 0, 4);
    return BSW_OK;
}

static int stage_chunk(Slot &s, const SeqPair *pairs, const uint8_t *ref, const uint8_t *qer, int32_t n,
                       const BlkStat *bs, int32_t nblk, bool two_bit, StagedChunk &c)
{
    int64_t r_lo = INT64_MAX, r_hi = 0, q_lo = INT64_MAX, q_hi = 0, r_sum = 0, q_sum = 0;
    for (int32_t b = 0; b < nblk; ++b) {
        r_lo = std::min(r_lo, bs[b].r_lo); r_hi = std::max(r_hi, bs[b].r_hi); r_sum += bs[b].r_sum;
        q_lo = std::min(q_lo, bs[b].q_lo); q_hi = std::max(q_hi, bs[b].q_hi); q_sum += bs[b].q_sum;
    }
    if (r_lo == INT64_MAX) r_lo = r_hi = 0;
    if (q_lo == INT64_MAX) q_lo = q_hi = 0;
    // bulk when the extents hold little besides the chunk's own bytes; else gather
    const bool bulk = (r_hi - r_lo) <= r_sum + r_sum / 4 + 4096 && (q_hi - q_lo) <= q_sum + q_sum / 4 + 4096;
    c.rb = (size_t)(bulk ? r_hi - r_lo : r_sum);
    c.qb = (size_t)(bulk ? q_hi - q_lo : q_sum);
    c.packed = bulk;
    c.n = n;
    if (bulk && two_bit && c.rb < ((size_t)1 << 30) && c.qb < ((size_t)1 << 30)) {
        const int r = stage_2bit(s, pairs, ref + r_lo, qer + q_lo, n, c);
        if (r != 1) {                       // 1: too many exception bytes -> nibbles below
            c.r_base = r_lo; c.q_base = q_lo;
            return r;
        }
    }
    c.mode = bulk ? kStageNibble : kStageGather;
    const size_t rs = bulk ? (c.rb + 1) / 2 : c.rb, qs = bulk ? (c.qb + 1) / 2 : c.qb;   // staged sizes
    c.n = n;
    c.pair_off = 0;
    c.ref_off = ((size_t)n * sizeof(SeqPair) + 255) & ~(size_t)255;
    c.qer_off = (c.ref_off + rs + 4 + 255) & ~(size_t)255;     // +4: kernels' aligned dword loads
    c.bytes = c.qer_off + qs + 4;
    if (c.bytes > s.cap_stage) {
        const size_t cap = std::max(c.bytes + c.bytes / 4, s.cap_stage * 3 / 2);
        if (s.h_stage) (void)hipHostFree(s.h_stage);
        s.h_stage = nullptr; s.cap_stage = 0;
        BSW_TRY(hipHostMalloc(&s.h_stage, cap, 0));
        s.cap_stage = cap;
    }
    uint8_t *h = (uint8_t *)s.h_stage;
    SeqPair *sp = (SeqPair *)(h + c.pair_off);
    if (bulk) {
        c.r_base = r_lo; c.q_base = q_lo;
        // records + both packs as one pool job list (pieces of ~2 MB)
        const size_t pb = (size_t)n * sizeof(SeqPair);
        const int np = (int)std::max<size_t>(1, pb >> 21), nr = (int)std::max<size_t>(1, c.rb >> 22),
                  nq = (int)std::max<size_t>(1, c.qb >> 22);
        auto even = [](size_t total, int k, int parts) {
            return k == parts ? total : (total * (size_t)k / (size_t)parts) & ~(size_t)31;
        };
        HostPool::get().parallel_for(np + nr + nq, [&](int t) {
            if (t < np) {
                const size_t a0 = pb * t / np, a1 = pb * (t + 1) / np;
                memcpy((char *)sp + a0, (const char *)pairs + a0, a1 - a0);
            } else if (t < np + nr) {
                const size_t a0 = even(c.rb, t - np, nr), a1 = even(c.rb, t - np + 1, nr);
                pack_nibbles(h + c.ref_off + a0 / 2, ref + r_lo + a0, a1 - a0);
            } else {
                const size_t a0 = even(c.qb, t - np - nr, nq), a1 = even(c.qb, t - np - nr + 1, nq);
                pack_nibbles(h + c.qer_off + a0 / 2, qer + q_lo + a0, a1 - a0);
            }
        });
    } else {
        par_memcpy(sp, pairs, (size_t)n * sizeof(SeqPair));
        c.r_base = c.q_base = 0;
        int64_t ro = 0, qo = 0;
        for (int32_t i = 0; i < n; ++i) {
            SeqPair &p = sp[i];
            if (p.len1 > 0) { memcpy(h + c.ref_off + ro, ref + p.idr, (size_t)p.len1); p.idr = (int32_t)ro; ro += p.len1; }
            else p.idr = 0;
            if (p.len2 > 0) { memcpy(h + c.qer_off + qo, qer + p.idq, (size_t)p.len2); p.idq = (int32_t)qo; qo += p.len2; }
            else p.idq = 0;
        }
    }
    memset(h + c.ref_off + rs, 0, 4);
    memset(h + c.qer_off + qs, 0, 4);
    return BSW_OK;
}

// outputs of a finished chunk (staged records) -> the caller's records.  Bulk-staged records
// carry the caller's own input fields, so whole records copy back; gathered ones had their
// offsets rewritten and copy field by field.
static void unstage_outputs(const Slot &s, SeqPair *pairs, int32_t n, int mode)
{
    if (mode == kStage2bit) {                           // 24 B of outputs per pair
        const int32_t *o = (const int32_t *)s.h_stage;
        const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(HostPool::workers() + 1, n >> 15));
        HostPool::get().parallel_for(nt, [&](int t) {
            for (int32_t i = (int32_t)((int64_t)n * t / nt); i < (int32_t)((int64_t)n * (t + 1) / nt); ++i) {
                const int32_t *q = o + 6 * (int64_t)i;
                pairs[i].score = q[0]; pairs[i].tle = q[1]; pairs[i].gtle = q[2];
                pairs[i].qle = q[3]; pairs[i].gscore = q[4]; pairs[i].max_off = q[5];
            }
        });
        return;
    }
    const SeqPair *sp = (const SeqPair *)s.h_stage;
    if (mode == kStageNibble) {
        par_memcpy(pairs, sp, (size_t)n * sizeof(SeqPair));
        return;
    }
    for (int32_t i = 0; i < n; ++i) {
        pairs[i].score = sp[i].score; pairs[i].tle = sp[i].tle; pairs[i].gtle = sp[i].gtle;
        pairs[i].qle = sp[i].qle; pairs[i].gscore = sp[i].gscore; pairs[i].max_off = sp[i].max_off;
    }
}

// The largest buffers any chunk of a host-buffer call needs, in the staging form stage_chunk will
// pick for it (2-bit for bulk extents, gathered bytes otherwise; a chunk that falls back to nibbles
// -- more than 1/32 non-ACGT bytes -- grows its slot as before): reserve_slot grows a slot to them
// before its first chunk.
struct SlotReserve {
    int32_t m = 0;                      // pairs
    size_t rb = 0, qb = 0, stage = 0;   // unpacked ref / qer bytes, pinned / device staging bytes
    void add(int32_t mc, const BlkStat *b, int32_t nb, bool two_bit)
    {
        int64_t r_lo = INT64_MAX, r_hi = 0, q_lo = INT64_MAX, q_hi = 0, r_sum = 0, q_sum = 0;
        for (int32_t k = 0; k < nb; ++k) {
            r_lo = std::min(r_lo, b[k].r_lo); r_hi = std::max(r_hi, b[k].r_hi); r_sum += b[k].r_sum;
            q_lo = std::min(q_lo, b[k].q_lo); q_hi = std::max(q_hi, b[k].q_hi); q_sum += b[k].q_sum;
        }
        if (r_lo == INT64_MAX) r_lo = r_hi = 0;
        if (q_lo == INT64_MAX) q_lo = q_hi = 0;
        // stage_chunk's choice: bulk when the extents hold little besides the chunk's own bytes
        const bool bulk = (r_hi - r_lo) <= r_sum + r_sum / 4 + 4096 && (q_hi - q_lo) <= q_sum + q_sum / 4 + 4096;
        const size_t r = (size_t)(bulk ? r_hi - r_lo : r_sum), q = (size_t)(bulk ? q_hi - q_lo : q_sum);
        const size_t mm = (size_t)mc;
        size_t st;
        if (bulk && two_bit && r < ((size_t)1 << 30) && q < ((size_t)1 << 30))
            st = std::max(align256(align256(align256(mm * sizeof(PairIn)) + (r + 3) / 4 + 4) + (q + 3) / 4 + 4) +
                              ((r + q) / 32 + 1024) * 4,
                          mm * 24);
        else if (bulk)
            st = align256(align256(mm * sizeof(SeqPair)) + (r + 1) / 2 + 4) + (q + 1) / 2 + 4;
        else
            st = align256(align256(mm * sizeof(SeqPair)) + r + 4) + q + 4;
        m = std::max(m, mc);
        rb = std::max(rb, r);
        qb = std::max(qb, q);
        stage = std::max(stage, st);
    }
};

static int reserve_slot(Slot &s, const SlotReserve &r)
{
    if (r.m <= 0) return BSW_OK;
    BSW_TRY(hipSetDevice(s.device));
    // the helper stream now, on the calling thread: created lazily by the enqueuer thread it cost
    // ~10 ms per slot (hipStreamCreateWithPriority) in the middle of a call's pipeline, stalling
    // every chunk queued behind it (HIP API trace, profiles/r06/hostpath_first_calls_api.txt)
    if (int e = ensure_pstream(s)) return e;
    if (r.stage > s.cap_stage) {
        if (s.h_stage) (void)hipHostFree(s.h_stage);
        s.h_stage = nullptr;
        s.cap_stage = 0;
        const size_t cap = r.stage + r.stage / 4;
        BSW_TRY(hipHostMalloc(&s.h_stage, cap, 0));
        s.cap_stage = cap;
    }
    BSW_TRY(grow(s.d_stage, s.cap_dstage, r.stage));
    BSW_TRY(grow(s.d_ref, s.cap_ref, r.rb + 16));
    BSW_TRY(grow(s.d_qer, s.cap_qer, r.qb + 16));
    BSW_TRY(grow(s.d_pairs, s.cap_pairs, (size_t)r.m));
    BSW_TRY(grow(s.d_bkt, s.cap_bkt, exc_buckets((int64_t)r.rb, (int64_t)r.qb)));
    BSW_TRY(grow_sort(s, r.m));
    size_t tmp_bytes = 0;
    BSW_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, s.d_keys, s.d_keys2, s.d_vals, s.d_order, r.m, 0,
                                               kKeyBits, (hipStream_t)0));
    BSW_TRY(grow(s.d_tmp, s.cap_tmp, tmp_bytes));
    return BSW_OK;
}

// Copy-engine warm-up, once per device context, on its first multi-chunk host call: H2D and D2H
// copies in flight at once on every slot's helper and DP streams, large and small, as the
// pipeline issues them.  Without it one hipMemcpyAsync in each of a context's first two calls
// blocked for 7.6-9.6 ms with the GPU idle (HIP API trace, profiles/r06/hostpath_first_calls_api.txt);
// with SDMA disabled (HSA_ENABLE_SDMA=0, blit-kernel copies) the stall was gone, so the first
// copies that land on a not yet used DMA engine pay its set-up.
static int prime_copies(Slot *const *slots, int ns)
{
    for (size_t want : {(size_t)1 << 62, (size_t)4 << 20, (size_t)64 << 10}) {
        for (int k = 0; k < ns; ++k) {
            Slot &s = *slots[k];
            const size_t half = std::min(s.cap_stage, s.cap_dstage) / 2, sz = std::min(want, half);
            if (sz == 0) continue;
            uint8_t *h = (uint8_t *)s.h_stage;
            BSW_TRY(hipMemcpyAsync(s.d_stage, h, sz, hipMemcpyHostToDevice, s.pstream));
            BSW_TRY(hipMemcpyAsync(h + half, s.d_stage + half, sz, hipMemcpyDeviceToHost, s.stream));
        }
        for (int k = 0; k < ns; ++k) {
            BSW_TRY(hipStreamSynchronize(slots[k]->pstream));
            BSW_TRY(hipStreamSynchronize(slots[k]->stream));
        }
    }
    return BSW_OK;
}

// One device's share of a host-buffer call: a pipeline of chunks over the device's slots (four by default).
// Per chunk: stage into the slot's pinned buffer (records + nibble-packed sequences, host
// pool) -> one H2D -> unpack -> plan / sort -> DP kernels -> D2H of the records.  The calling
// thread only stages and enqueues copies and plans; a launcher thread enqueues each chunk's DP
// kernels and record readback as soon as that chunk's class counts are back, so the GPU never
// waits for the host to finish staging the next chunk (round 1's single-thread loop launched
// chunk k's kernels only after chunk k + 1 was staged: ~1.4 ms of idle GPU per chunk in the
// rocprofv3 timeline).  Chunks ramp from ~n/32 pairs up to `chunk` so the first kernels start
// early.  Outputs are identical to one unchunked call (pairs are independent).
static int host_shard(const KParams &kp, DeviceCtx &dc, SeqPair *pairs, const uint8_t *ref,
                      const uint8_t *qer, int32_t n, int32_t w, int cell_bits, int32_t chunk, bool two_bit,
                      bsw_stats_t *st)
{
    if (n == 0) return BSW_OK;
    auto now = [] { return std::chrono::steady_clock::now(); };
    const auto t_start = now();
    // the whole prepass (validation + per-block byte extents) before chunk 0: validating only chunk
    // 0's blocks first and the rest after it started measured no faster
    std::vector<BlkStat> bs;
    if (!prepass(pairs, n, bs)) return BSW_E_RANGE;
    if (chunk <= 0) chunk = n;
    // slots are taken as chunks start (a one-chunk call takes one); chunk k + nslots stages only
    // once chunk k's outputs are back.  4 since round 4: with the helper stream the fourth slot
    // lets the next chunk stage a DP generation earlier (same box, alternating: 84.7 / 87.7 vs
    // 77.0 / 78.8 M/s per 1M-pair call; 5 slots pay more first-call allocation,
    // profiles/r04/hostpath_slots_r4w.txt)
#ifndef BSW_HP_SLOTS                   // experiment builds only (make abhost AB_FLAGS=-DBSW_HP_SLOTS=5)
#define BSW_HP_SLOTS 4
#endif
    constexpr int nslots = BSW_HP_SLOTS;
    int rc = BSW_OK;
    std::unique_ptr<Slot> slots[nslots];
    slots[0] = dc.acquire(rc);
    if (rc) return rc;
    int32_t pend_at[nslots] = {}, pend_n[nslots] = {};  // chunk in flight per slot
    int32_t pend_seq[nslots];
    std::fill(pend_seq, pend_seq + nslots, -1);
    int pend_mode[nslots] = {};
    bsw_stats_t agg{};
    // Everything but the DP kernels runs on the slot's high-priority stream: the next chunk's
    // copies, unpack / plan / sort kernels and the outputs' readback are dispatched ahead of the
    // queued DP workgroups instead of behind them
    // launcher thread: chunk seq numbers in order; launched[k] = last seq whose DP is enqueued
    struct Launcher {
        std::mutex mu;
        std::condition_variable cv;
        struct Job { int first; int32_t second; int mode; };
        std::deque<Job> q;                        // (slot, seq, staging mode)
        int32_t launched[nslots];
        bool stop = false;
        int rc = BSW_OK;
    } L;
    std::fill(L.launched, L.launched + nslots, -1);
    std::thread launcher([&] {
        const bool dev_ok = hipSetDevice(dc.device) == hipSuccess;
        for (;;) {
            Launcher::Job job;
            {
                std::unique_lock<std::mutex> lk(L.mu);
                L.cv.wait(lk, [&] { return L.stop || !L.q.empty(); });
                if (L.q.empty()) return;
                job = L.q.front();
                L.q.pop_front();
            }
            int r = dev_ok ? BSW_OK : BSW_E_HIP;
            {
                std::lock_guard<std::mutex> g(L.mu);
                if (L.rc) r = L.rc;
            }
            Slot &p = *slots[job.first];
            if (!r) r = run_dp(kp, p);
            // the outputs' gather and readback go on the high-priority stream once the DP (and its
            // guard readback) is done: on the DP stream they would queue behind the next chunks'
            // DP workgroups (a 1.4 ms copy in the trace)
            hipStream_t os = p.run_stream;
            hipStream_t hs = p.plan.plan_stream;       // the chunk's helper stream
            if (!r && hs && p.run_stream != hs) {
                if (!p.evd && hipEventCreateWithFlags(&p.evd, hipEventDisableTiming) != hipSuccess) r = BSW_E_HIP;
                if (!r && (hipEventRecord(p.evd, p.run_stream) != hipSuccess ||
                           hipStreamWaitEvent(hs, p.evd, 0) != hipSuccess))
                    r = BSW_E_HIP;
                os = hs;
                p.run_stream = hs;                     // finish_stats waits here: after the DP's stream
            }
            if (!r && job.mode == kStage2bit) {        // outputs only: 24 B per pair
                const int32_t m = p.plan.n;
                hipLaunchKernelGGL(gather_outputs_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, os,
                                   p.plan.d_pairs, (int32_t *)p.d_stage, m);
                if (hipGetLastError() != hipSuccess ||
                    hipMemcpyAsync(p.h_stage, p.d_stage, (size_t)m * 24, hipMemcpyDeviceToHost, os) != hipSuccess)
                    r = BSW_E_HIP;
            } else if (!r && hipMemcpyAsync(p.h_stage, p.plan.d_pairs, (size_t)p.plan.n * sizeof(SeqPair),
                                            hipMemcpyDeviceToHost, os) != hipSuccess) {
                r = BSW_E_HIP;
            }
            {
                std::lock_guard<std::mutex> g(L.mu);
                if (r && !L.rc) L.rc = r;
                L.launched[job.first] = job.second;
            }
            L.cv.notify_all();
        }
    });
    auto stop_launcher = [&] {
        {
            std::lock_guard<std::mutex> g(L.mu);
            L.stop = true;
        }
        L.cv.notify_all();
        if (launcher.joinable()) launcher.join();
    };
    auto finish = [&](int k) -> int {                   // wait for slot k's chunk, outputs back
        if (pend_n[k] == 0) return BSW_OK;
        {
            std::unique_lock<std::mutex> lk(L.mu);
            L.cv.wait(lk, [&] { return L.launched[k] == pend_seq[k]; });
            if (L.rc) return L.rc;
        }
        Slot &s = *slots[k];
        const int r = finish_stats(s);                  // also BSW_E_RANGE: kernel guard tripped
        if (r) return r;
        unstage_outputs(s, pairs + pend_at[k], pend_n[k], pend_mode[k]);
        agg.kernel_ms += s.stats.kernel_ms;
        agg.n_i16 += s.stats.n_i16; agg.n_u8 += s.stats.n_u8; agg.n_wide += s.stats.n_wide;
        agg.n_packed += s.stats.n_packed; agg.n_launches += s.stats.n_launches; agg.n_wave += s.stats.n_wave; agg.n_group += s.stats.n_group;
        pend_n[k] = 0;
        return BSW_OK;
    };
    // the device side of one staged chunk -- H2D of the slot's staging buffer, unpack kernels,
    // plan / sort -- then its launcher job.  On a failure the job still goes to the launcher,
    // which skips its DP and releases finish(k) with the error
    auto enqueue = [&](int k, int32_t seq, const StagedChunk &c, int32_t m) -> int {
        Slot &s = *slots[k];
        const int r = [&]() -> int {
            if (int e = ensure_pstream(s)) return e;
            hipStream_t hs = s.pstream;
            BSW_TRY(grow(s.d_stage, s.cap_dstage, c.bytes));
            BSW_TRY(hipMemcpyAsync(s.d_stage, s.h_stage, c.bytes, hipMemcpyHostToDevice, hs));
            const uint8_t *d_r = s.d_stage + c.ref_off, *d_q = s.d_stage + c.qer_off;
            SeqPair *d_p = (SeqPair *)(s.d_stage + c.pair_off);
            if (c.mode == kStage2bit) {     // 2-bit codes -> bytes, exceptions patched, records expanded
                // one launch (stage_in_kernel: both unpacks, the exception patches, the records and
                // the pad zeroing) instead of six: a chunk's enqueue is launch-bound on the host
                // (~60 us per launch while the pool packs the next chunk, HIP API trace
                // profiles/r04/hostpath_api_trace.txt)
                BSW_TRY(grow(s.d_ref, s.cap_ref, c.rb + 16));
                BSW_TRY(grow(s.d_qer, s.cap_qer, c.qb + 16));
                BSW_TRY(grow(s.d_pairs, s.cap_pairs, (size_t)m));
                if (int e = launch_stage_in(s, hs, s.d_stage + c.ref_off, (int64_t)c.rb, s.d_stage + c.qer_off,
                                            (int64_t)c.qb, (const uint32_t *)(s.d_stage + c.exc_off), c.n_exr,
                                            c.n_exr + c.n_exq, (const PairIn *)(s.d_stage + c.pair_off), m, s.d_ref,
                                            s.d_qer, s.d_pairs, nullptr))
                    return e;
                d_r = s.d_ref;
                d_q = s.d_qer;
                d_p = s.d_pairs;
            } else if (c.packed) {          // nibbles -> one byte per base in the slot's buffers
                BSW_TRY(grow(s.d_ref, s.cap_ref, c.rb + 4));
                BSW_TRY(grow(s.d_qer, s.cap_qer, c.qb + 4));
                BSW_TRY(hipMemsetAsync(s.d_ref + c.rb, 0, 4, hs));
                BSW_TRY(hipMemsetAsync(s.d_qer + c.qb, 0, 4, hs));
                const int64_t tr = ((int64_t)c.rb + 7) / 8, tq = ((int64_t)c.qb + 7) / 8;
                if (tr > 0)
                    hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)((tr + 255) / 256)), dim3(256), 0, hs,
                                       d_r, s.d_ref, (int64_t)c.rb);
                if (tq > 0)
                    hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)((tq + 255) / 256)), dim3(256), 0, hs,
                                       d_q, s.d_qer, (int64_t)c.qb);
                BSW_TRY(hipGetLastError());
                d_r = s.d_ref;
                d_q = s.d_qer;
            }
            PlanCall pc;
            pc.d_pairs = d_p;
            // kernels index ref / qer by idr / idq: shift the bases so staged byte 0 is r_base / q_base
            pc.d_ref = d_r - c.r_base;
            pc.d_qer = d_q - c.q_base;
            pc.n = m; pc.w = w; pc.cell_bits = cell_bits; pc.stream = hs;
            pc.dp_stream = s.stream;
            pc.plan_stream = hs;
            return run_plan(kp, s, pc);
        }();
        {
            std::lock_guard<std::mutex> g(L.mu);
            if (r && !L.rc) L.rc = r;
            L.q.push_back(Launcher::Job{k, seq, c.mode});
        }
        L.cv.notify_all();
        return r;
    };
    // Calls of several chunks hand each staged chunk to an enqueuer thread, so the calling thread
    // stages the next chunk at once: the enqueue of a chunk (H2D, unpack, plan, sort -- ~0.9 ms
    // of runtime calls per 256K-pair chunk in the kernel + copy trace) otherwise sat between two
    // stagings and made the next chunk's DP start after the current one had drained
    // (profiles/r04/hostpath_trace_*.txt).  One-chunk calls enqueue inline (no thread hand-off).
    struct EnqJob { int k; int32_t seq; StagedChunk c; int32_t m; };
    struct Enqueuer {
        std::mutex mu;
        std::condition_variable cv;
        std::deque<EnqJob> q;
        bool stop = false;
    } E;
    const int32_t nblk0 = (int32_t)bs.size();
    // the first chunk: 16 blocks (64K pairs) or 1/32 of the call.  The same size decides whether
    // the call runs as several chunks (enqueuer thread) and cuts the chunks below
#ifndef BSW_HP_FIRST_BLK               // experiment builds only (make abhost AB_FLAGS=-DBSW_HP_FIRST_BLK=8)
#define BSW_HP_FIRST_BLK 16
#endif
    const int32_t first_blk = std::min(std::max<int32_t>(1, chunk / kStageBlk),
                                       nblk0 <= 32 ? nblk0 : std::max<int32_t>(BSW_HP_FIRST_BLK, nblk0 / 32));
    const bool async = nblk0 > first_blk;
    std::thread enqueuer;
    if (async)
        enqueuer = std::thread([&] {
            const bool dev_ok = hipSetDevice(dc.device) == hipSuccess;
            for (;;) {
                EnqJob job;
                {
                    std::unique_lock<std::mutex> lk(E.mu);
                    E.cv.wait(lk, [&] { return E.stop || !E.q.empty(); });
                    if (E.q.empty()) return;
                    job = E.q.front();
                    E.q.pop_front();
                }
                if (!dev_ok) {
                    std::lock_guard<std::mutex> g(L.mu);
                    if (!L.rc) L.rc = BSW_E_HIP;
                    L.q.push_back(Launcher::Job{job.k, job.seq, job.c.mode});
                    L.cv.notify_all();
                    continue;
                }
                (void)enqueue(job.k, job.seq, job.c, job.m);
            }
        });
    auto stop_enqueuer = [&] {
        {
            std::lock_guard<std::mutex> g(E.mu);
            E.stop = true;
        }
        E.cv.notify_all();
        if (enqueuer.joinable()) enqueuer.join();
    };
    double stage_ms = 0;
    // the chunk schedule (block ranges): `cur` blocks, doubling from first_blk up to `chunk` pairs,
    // fewer when their sequence bytes pass ~512 MB (staged offsets stay int32).  (A small remainder
    // stays its own chunk: folded into the last full chunk it added a third, nearly empty generation
    // of waves to that launch -- 262144 pairs are exactly two generations at two waves per SIMD --
    // and the call got ~1 ms slower; as its own launch it runs beside the last chunk on another
    // queue.  Measured)  Calls of up to 128K pairs -- kt_for-sized batches -- run as
    // one chunk on one slot.
    std::vector<std::pair<int32_t, int32_t>> chs;
    SlotReserve res{};
    {
        const int32_t nblk = (int32_t)bs.size();
        const int32_t cap_blk = std::max<int32_t>(1, chunk / kStageBlk);
        for (int32_t b = 0, nb = 0, cur = first_blk; b < nblk; b += nb, cur = std::min(cap_blk, cur * 2)) {
            int64_t bytes = 0;
            for (nb = 0; nb < cur && b + nb < nblk; ++nb) {
                const int64_t x = bs[b + nb].r_sum + bs[b + nb].q_sum;
                if (nb > 0 && bytes + x > ((int64_t)1 << 29)) break;
                bytes += x;
            }
            chs.emplace_back(b, nb);
            res.add(std::min(n, (b + nb) * kStageBlk) - b * kStageBlk, bs.data() + b, nb, two_bit);
        }
    }

    rc = [&]() -> int {
        BSW_TRY(hipSetDevice(dc.device));
        if (int r = reserve_slot(*slots[0], res)) return r;     // (slot 0 was taken before the schedule)
        if (chs.size() > 1 && !dc.copies_warm.exchange(true)) {
            // the context's first pipelined call: every slot it will use now, then the copy
            // warm-up over all of them at once (prime_copies)
            const int ns = std::min<int>(nslots, (int)chs.size());
            Slot *sp[nslots] = {slots[0].get()};
            for (int j = 1; j < ns; ++j) {
                int r = BSW_OK;
                slots[j] = dc.acquire(r);
                if (r) return r;
                if ((r = reserve_slot(*slots[j], res))) return r;
                sp[j] = slots[j].get();
            }
            if (int r = prime_copies(sp, ns)) return r;
        }
        int k = 0;
        int32_t seq = 0;
        for (const auto &ch : chs) {
            const int32_t b = ch.first, nb = ch.second;
            const int32_t a = b * kStageBlk, m = std::min(n, (b + nb) * kStageBlk) - a;
            int r = finish(k);                          // slot k's last chunk
            if (r) return r;
            if (!slots[k]) {
                slots[k] = dc.acquire(r);
                if (r) return r;
                // every buffer of the slot at the call's largest chunk at once: chunks rotate over
                // the slots, so sizing by the chunk at hand regrew a slot (hipFree waits for the
                // device) on the first calls of a context as its chunks got larger
                if ((r = reserve_slot(*slots[k], res))) return r;
            }
            Slot &s = *slots[k];
            StagedChunk c;
            const auto t0 = now();
            if ((r = stage_chunk(s, pairs + a, ref, qer, m, bs.data() + b, nb, two_bit, c))) return r;
            stage_ms += std::chrono::duration<double, std::milli>(now() - t0).count();
            pend_at[k] = a; pend_n[k] = m; pend_mode[k] = c.mode; pend_seq[k] = seq;
            if (async) {
                {
                    std::lock_guard<std::mutex> g(E.mu);
                    E.q.push_back(EnqJob{k, seq, c, m});
                }
                E.cv.notify_all();
            } else if ((r = enqueue(k, seq, c, m))) {
                return r;
            }
            k = (k + 1) % nslots;
            ++seq;
        }
        for (int j = 0; j < nslots; ++j) {
            const int r = finish(j);
            if (r) return r;
        }
        return BSW_OK;
    }();
    stop_enqueuer();                                    // drains its queue first (every job reaches the launcher)
    stop_launcher();                                    // drains the queue first (it exits only when empty)
    agg.stage_ms = (float)stage_ms;
    agg.host_ms = (float)std::chrono::duration<double, std::milli>(now() - t_start).count();
    for (int k = 0; k < nslots; ++k) {
        if (!slots[k]) continue;
        if (rc) {                                       // nothing in flight on a returned slot
            (void)hipStreamSynchronize(slots[k]->stream);
            if (slots[k]->pstream) (void)hipStreamSynchronize(slots[k]->pstream);
        }
        dc.give_back(std::move(slots[k]));
    }
    if (rc == BSW_OK && st) *st = agg;
    return rc;
}

// ---------------------------------------------------------------- cross-call coalescing
// Upstream's kt_for workers each hand getScores* a few thousand pairs per call.  Run one by one,
// every such call pays a plan / sort / DP launch sequence whose lane-per-pair waves live ~1 ms
// whatever the batch size, and 8 workers' calls contend for the runtime.  Here a small call
// (<= BSW_OPT_COALESCE pairs) is queued on its device; the first caller that finds fewer than
// agg_leaders_max batches in flight becomes a leader, takes EVERY queued call of the same
// (w, cell_bits, end_bonus) -- its own or others' -- and runs them as one device batch: the
// callers' contiguous byte extents 2-bit-packed side by side in one pinned staging buffer
// (records rebased), one H2D, one plan / sort / DP, 24 B of outputs per pair back, scattered
// to each caller's records.  A lone caller leads its own one-call batch at once (no added
// wait); under load, calls that arrive while a batch is on the GPU form the next one.
// Outputs are identical to separate calls (pairs are independent).
struct AggReq {
    SeqPair *pairs;
    const uint8_t *ref, *qer;
    int32_t n, w;
    int cell_bits;
    int32_t eb;
    int rc = BSW_OK;
    bsw_stats_t st{};
    bool done = false;
};
constexpr int32_t kAggMaxPairs = 262144;        // pairs per coalesced batch
constexpr int64_t kAggLingerPairs = 4096;       // a lingering leader starts once this many are queued

struct AggSeg {                                 // one call inside a coalesced batch
    AggReq *r;
    int64_t r_lo, r_hi, q_lo, q_hi;             // the call's byte extents in its own buffers
    int64_t r_off, q_off;                       // their offsets in the batch's code space
    int32_t p_off;                              // first record in the batch
};

static int run_group_staged(const KParams &kp, DeviceCtx &dc, std::vector<AggSeg> &segs, int32_t N, int64_t r_tot,
                            int64_t q_tot, int32_t w, int cell_bits, bsw_stats_t &st)
{
    int rc = BSW_OK;
    auto slot = dc.acquire(rc);
    if (!slot) return rc;
    Slot &s = *slot;
    rc = [&]() -> int {
        BSW_TRY(hipSetDevice(dc.device));
        const size_t rs = (size_t)(r_tot + 3) / 4, qs = (size_t)(q_tot + 3) / 4;
        const size_t exc_cap = (size_t)(r_tot + q_tot) / 32 + 1024;
        const size_t pair_off = 0, ref_off = align256((size_t)N * sizeof(PairIn));
        const size_t qer_off = align256(ref_off + rs + 4), exc_off = align256(qer_off + qs + 4);
        const size_t bytes = std::max(exc_off + exc_cap * 4, (size_t)N * 24);
        if (bytes > s.cap_stage) {
            const size_t cap = std::max(bytes + bytes / 4, s.cap_stage * 3 / 2);
            if (s.h_stage) (void)hipHostFree(s.h_stage);
            s.h_stage = nullptr; s.cap_stage = 0;
            BSW_TRY(hipHostMalloc(&s.h_stage, cap, 0));
            s.cap_stage = cap;
        }
        const auto tg0 = std::chrono::steady_clock::now();
        uint8_t *h = (uint8_t *)s.h_stage;
        memset(h + ref_off, 0, rs + 4);                 // the padding between calls' extents
        memset(h + qer_off, 0, qs + 4);
        // tasks: per call its records, and its ref / qer extents in pieces of <= 1 MB cut at
        // multiples of 64 codes (every call's extent starts 64-aligned in the code space)
        struct Task { int seg, kind; int64_t a, b; };
        std::vector<Task> tasks;
        constexpr int64_t kPiece = (int64_t)1 << 20;
        for (int g = 0; g < (int)segs.size(); ++g) {
            tasks.push_back(Task{g, 0, 0, 0});
            for (int kind = 1; kind <= 2; ++kind) {
                const int64_t len = kind == 1 ? segs[g].r_hi - segs[g].r_lo : segs[g].q_hi - segs[g].q_lo;
                for (int64_t a = 0; a < len; a += kPiece) tasks.push_back(Task{g, kind, a, std::min(len, a + kPiece)});
            }
        }
        std::vector<std::vector<uint32_t>> ex(tasks.size());
        // per task: the row-group kernel's contract over its records (max qlen, or -1: a misfit)
        std::vector<int> gq_maxq(tasks.size(), 0), gq_maxt(tasks.size(), 0);
        PairIn *pin = (PairIn *)(h + pair_off);
        HostPool::get().parallel_for((int)tasks.size(), [&](int t) {
            const Task &k = tasks[t];
            const AggSeg &g = segs[k.seg];
            if (k.kind == 0) {
                const SeqPair *p = g.r->pairs;
                int maxq = 0, maxt = 0;
                for (int32_t i = 0; i < g.r->n; ++i) {
                    PairIn &o = pin[g.p_off + i];
                    o.idr = p[i].len1 > 0 ? (int32_t)(p[i].idr - g.r_lo + g.r_off) : 0;
                    o.idq = p[i].len2 > 0 ? (int32_t)(p[i].idq - g.q_lo + g.q_off) : 0;
                    o.len1 = p[i].len1; o.len2 = p[i].len2; o.h0 = p[i].h0;
                    if (maxq >= 0) maxq = gq_pair_ok(kp, p[i].len2, p[i].len1, p[i].h0, 16) ? std::max(maxq, p[i].len2) : -1;
                    maxt = std::max(maxt, p[i].len1);
                }
                gq_maxq[t] = maxq;
                gq_maxt[t] = maxt;
            } else if (k.kind == 1) {
                pack_2bit(h + ref_off + (g.r_off + k.a) / 4, g.r->ref + g.r_lo + k.a, (size_t)(k.b - k.a),
                          (uint32_t)(g.r_off + k.a), ex[t]);
            } else {
                pack_2bit(h + qer_off + (g.q_off + k.a) / 4, g.r->qer + g.q_lo + k.a, (size_t)(k.b - k.a),
                          (uint32_t)(g.q_off + k.a), ex[t]);
            }
        });
        size_t n_r = 0, n_q = 0;
        for (size_t t = 0; t < tasks.size(); ++t) (tasks[t].kind == 1 ? n_r : n_q) += ex[t].size();
        if (n_r + n_q > exc_cap) return 1;              // too many non-ACGT bytes: caller splits
        uint32_t *exw = (uint32_t *)(h + exc_off);
        size_t o_r = 0, o_q = n_r;
        for (size_t t = 0; t < tasks.size(); ++t) {
            if (ex[t].empty()) continue;
            size_t &o = tasks[t].kind == 1 ? o_r : o_q;
            memcpy(exw + o, ex[t].data(), ex[t].size() * 4);
            o += ex[t].size();
        }
        const size_t up = exc_off + (n_r + n_q) * 4;
        const auto tg1 = std::chrono::steady_clock::now();
        BSW_TRY(grow(s.d_stage, s.cap_dstage, std::max(up, (size_t)N * 24)));
        BSW_TRY(hipMemcpyAsync(s.d_stage, s.h_stage, up, hipMemcpyHostToDevice, s.stream));
        BSW_TRY(grow(s.d_ref, s.cap_ref, (size_t)r_tot + 4));
        BSW_TRY(grow(s.d_qer, s.cap_qer, (size_t)q_tot + 4));
        BSW_TRY(grow(s.d_pairs, s.cap_pairs, (size_t)N));
        const int32_t ne = (int32_t)(n_r + n_q);
        if (int e = launch_stage_in(s, s.stream, s.d_stage + ref_off, r_tot, s.d_stage + qer_off, q_tot,
                                    (const uint32_t *)(s.d_stage + exc_off), (int32_t)n_r, ne,
                                    (const PairIn *)(s.d_stage + pair_off), N, s.d_ref, s.d_qer, s.d_pairs,
                                    s.d_meta + kMetaErr))
            return e;
        PlanCall pc;
        pc.d_pairs = s.d_pairs; pc.d_ref = s.d_ref; pc.d_qer = s.d_qer;
        pc.n = N; pc.w = w; pc.cell_bits = cell_bits; pc.stream = s.stream;
        int gq_max = 0, gq_mt = 0;
        for (size_t t = 0; t < tasks.size(); ++t)
            if (tasks[t].kind == 0) {
                gq_max = (gq_max < 0 || gq_maxq[t] < 0) ? -1 : std::max(gq_max, gq_maxq[t]);
                gq_mt = std::max(gq_mt, gq_maxt[t]);
            }
        pc.gq_maxq = gq_max;
        pc.gq_maxt = gq_mt;
        // host-checked row-group batch: the kernel writes the 24 output bytes per pair straight
        // into the staging buffer (its inputs were expanded out of it above)
        if (pc.gq_maxq >= 0) pc.d_out24 = (int32_t *)s.d_stage;
        int r = run_plan(kp, s, pc);
        if (!r) r = run_dp(kp, s);
        if (r) {
            (void)hipStreamSynchronize(s.stream);
            return r;
        }
        if (!(s.fast == 2 && s.plan.d_out24)) {
            hipLaunchKernelGGL(gather_outputs_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s.stream,
                               s.d_pairs, (int32_t *)s.d_stage, N);
            BSW_TRY(hipGetLastError());
        }
        BSW_TRY(hipMemcpyAsync(s.h_stage, s.d_stage, (size_t)N * 24, hipMemcpyDeviceToHost, s.stream));
        // the leader polls its batch (~0.3 ms) instead of the runtime's blocking wait: 8 callers x 1K
        // coalesced 11.4 / 12.4 -> 14.1 / 13.5 M/s (same box, alternating; profiles/r05/slot_ownq_percall.txt)
        if ((r = finish_stats(s, true))) return r;
        const int32_t *out = (const int32_t *)s.h_stage;
        auto scatter = [&](int g) {
            SeqPair *p = segs[g].r->pairs;
            const int32_t *q = out + 6 * (int64_t)segs[g].p_off;
            for (int32_t i = 0; i < segs[g].r->n; ++i, q += 6) {
                p[i].score = q[0]; p[i].tle = q[1]; p[i].gtle = q[2];
                p[i].qle = q[3]; p[i].gscore = q[4]; p[i].max_off = q[5];
            }
        };
        // a few thousand records: on this thread (waking the host pool costs more than the copy)
        if (N <= 16384)
            for (int g = 0; g < (int)segs.size(); ++g) scatter(g);
        else
            HostPool::get().parallel_for((int)segs.size(), scatter);
        st = s.stats;
        st.stage_ms = (float)std::chrono::duration<double, std::milli>(tg1 - tg0).count();
        return BSW_OK;
    }();
    dc.give_back(std::move(slot), rc);
    return rc;
}

// One coalesced batch: calls that fail validation get BSW_E_RANGE; calls whose buffers are not
// contiguous (scattered idr / idq) and batches with too many non-ACGT bytes run on their own
// through host_shard.
static void run_group(const KParams &kp, DeviceCtx &dc, std::vector<AggReq *> &G, int32_t chunk, bool two_bit)
{
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<AggSeg> segs;
    std::vector<AggReq *> alone;
    int64_t r_tot = 0, q_tot = 0;
    int32_t N = 0;
    for (AggReq *r : G) {
        std::vector<BlkStat> bs;
        if (!prepass(r->pairs, r->n, bs)) { r->rc = BSW_E_RANGE; continue; }
        int64_t r_lo = INT64_MAX, r_hi = 0, q_lo = INT64_MAX, q_hi = 0, r_sum = 0, q_sum = 0;
        for (const auto &b : bs) {
            r_lo = std::min(r_lo, b.r_lo); r_hi = std::max(r_hi, b.r_hi); r_sum += b.r_sum;
            q_lo = std::min(q_lo, b.q_lo); q_hi = std::max(q_hi, b.q_hi); q_sum += b.q_sum;
        }
        if (r_lo == INT64_MAX) r_lo = r_hi = 0;
        if (q_lo == INT64_MAX) q_lo = q_hi = 0;
        const bool bulk = (r_hi - r_lo) <= r_sum + r_sum / 4 + 4096 && (q_hi - q_lo) <= q_sum + q_sum / 4 + 4096;
        if (!two_bit || !bulk) { alone.push_back(r); continue; }
        segs.push_back(AggSeg{r, r_lo, r_hi, q_lo, q_hi, r_tot, q_tot, N});
        r_tot = (r_tot + (r_hi - r_lo) + 63) & ~(int64_t)63;
        q_tot = (q_tot + (q_hi - q_lo) + 63) & ~(int64_t)63;
        N += r->n;
    }
    if (!segs.empty()) {
        bsw_stats_t st{};
        const int rc = (r_tot < ((int64_t)1 << 30) && q_tot < ((int64_t)1 << 30))
                           ? run_group_staged(kp, dc, segs, N, r_tot, q_tot, segs[0].r->w, segs[0].r->cell_bits, st)
                           : 1;
        if (rc == 1) {
            for (auto &g : segs) alone.push_back(g.r);
        } else {
            st.n_devices = 1;
            st.host_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
            for (auto &g : segs) { g.r->rc = rc; g.r->st = st; }
        }
    }
    for (AggReq *r : alone) {
        bsw_stats_t st{};
        r->rc = host_shard(kp, dc, r->pairs, r->ref, r->qer, r->n, r->w, r->cell_bits, chunk, two_bit, &st);
        st.n_devices = 1;
        r->st = st;
    }
}

static int coalesced_call(const KParams &kp, DeviceCtx &dc, SeqPair *pairs, const uint8_t *ref, const uint8_t *qer,
                          int32_t n, int32_t w, int cell_bits, int32_t chunk, bool two_bit, bsw_stats_t *st)
{
    AggReq me{pairs, ref, qer, n, w, cell_bits, kp.end_bonus};
    std::unique_lock<std::mutex> lk(dc.agg_mu);
    dc.agg_q.push_back(&me);
    dc.agg_qn += n;
    ++dc.agg_inside;
    if (dc.agg_lingering > 0) dc.agg_cv.notify_all();      // a lingering leader counts the queue
    while (!me.done) {
        if (dc.agg_leaders < dc.agg_leaders_max && !dc.agg_q.empty()) {
            // lead: every queued call with the front call's (w, cell_bits, end_bonus), FIFO
            // linger only when there are more callers than leader slots (batching is then the only
            // way to serve them all) and two or more batches run: with fewer callers the batches
            // must overlap instead -- a lingering leader serialised 2 callers (1K: 4.0 vs 6.8 M/s)
            // and cost 4 callers a quarter (profiles/r04/percall_linger_r4{q,r}.txt)
            if (dc.agg_inside > dc.agg_leaders_max && dc.agg_nrun >= 2 && dc.agg_linger_us > 0 &&
                dc.agg_qn < kAggLingerPairs) {
                // the device is busy anyway: hold this leader's place until the queue holds
                // kAggLingerPairs pairs (the next calls of the callers whose batches just finished),
                // the device goes idle, or linger_us passes -- a row-group batch costs ~0.3 ms
                // whether it carries 1K or 4K pairs, so fuller batches are the small-call
                // throughput
                ++dc.agg_leaders;
                ++dc.agg_lingering;
                dc.agg_cv.wait_for(lk, std::chrono::microseconds(dc.agg_linger_us), [&] {
                    return me.done || dc.agg_qn >= kAggLingerPairs || dc.agg_nrun < 2;
                });
                --dc.agg_lingering;
                --dc.agg_leaders;
                if (me.done) break;
                if (dc.agg_q.empty()) continue;       // another leader took every queued call
            }
            ++dc.agg_leaders;
            std::vector<AggReq *> G;
            const AggReq *f = dc.agg_q.front();
            const int32_t fw = f->w, feb = f->eb;
            const int fcb = f->cell_bits;
            int64_t tot = 0;
            for (auto it = dc.agg_q.begin(); it != dc.agg_q.end();) {
                AggReq *r = *it;
                if (r->w == fw && r->cell_bits == fcb && r->eb == feb && (G.empty() || tot + r->n <= kAggMaxPairs)) {
                    G.push_back(r);
                    tot += r->n;
                    dc.agg_qn -= r->n;
                    it = dc.agg_q.erase(it);
                } else {
                    ++it;
                }
            }
            dc.agg_run += tot;
            ++dc.agg_nrun;
            lk.unlock();
            KParams gk = kp;
            gk.end_bonus = feb;
            run_group(gk, dc, G, chunk, two_bit);
            lk.lock();
            dc.agg_run -= tot;
            --dc.agg_nrun;
            --dc.agg_leaders;
            for (AggReq *r : G) r->done = true;
            dc.agg_cv.notify_all();
        } else {
            dc.agg_cv.wait(lk);
        }
    }
    --dc.agg_inside;
    if (st) *st = me.st;
    return me.rc;
}

// ---------------------------------------------------------------- mate rescue (bsw_mate.h)
static void make_mate_params(const bsw_params_t &p, MateParams &mp)
{
    memset(&mp, 0, sizeof(mp));
    mp.e_del = p.e_del; mp.oe_del = p.o_del + p.e_del;
    mp.e_ins = p.e_ins; mp.oe_ins = p.o_ins + p.e_ins;
    int mn = 127, mx = 0;                                 // ksw_qinit: min(mat, 127), max(mat, 0)
    for (int i = 0; i < 25; ++i) { mn = std::min(mn, (int)p.mat[i]); mx = std::max(mx, (int)p.mat[i]); }
    mp.maxsc = mx;
    mp.shift = (uint8_t)(256 - (uint8_t)(int8_t)mn);
    for (int t = 0; t < 5; ++t) {
        uint8_t b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int q = 0; q < 5; ++q) b[q] = (uint8_t)p.mat[t * 5 + q];
        memcpy(mp.prof[t], b, 8);
    }
}

static bool mate_params_ok(const bsw_params_t &p)
{
    int mx = 0;
    for (int i = 0; i < 25; ++i) mx = std::max(mx, (int)p.mat[i]);
    return p.o_ins >= 1 && mx >= 1;
}

// Forward pass (ksw_u8 / ksw_i16 per job) then, for jobs with KSW_XSTART, the reverse pass;
// each pass: device bucketing by (P, slen), one readback of the bucket ranges, one launch per
// ncol class.  Blocking.
static int mate_device(const MateParams &mp, Slot &s, const SeqPair *d_pairs, const uint8_t *d_ref,
                       const uint8_t *d_qer, int32_t n, bsw_kswr_t *d_aln, hipStream_t st,
                       bsw_mate_stats_t *stats)
{
    *stats = bsw_mate_stats_t{};
    const size_t jcap = (size_t)n + 64 * kMateBuckets;
    BSW_TRY(grow(s.d_mjobs, s.cap_mjobs, jcap));
    if (!s.d_mmeta) BSW_TRY(hipMalloc((void **)&s.d_mmeta, kMateMetaWords * sizeof(int32_t)));
    if (!s.h_mmeta) BSW_TRY(hipHostMalloc((void **)&s.h_mmeta, kMateMetaWords * sizeof(int32_t), 0));
    if (!s.d_mcells) BSW_TRY(hipMalloc((void **)&s.d_mcells, sizeof(unsigned long long)));
    if (!s.ev2) BSW_TRY(hipEventCreate(&s.ev2));
    if (!s.ev3) BSW_TRY(hipEventCreate(&s.ev3));
    BSW_TRY(hipMemsetAsync(s.d_mcells, 0, sizeof(unsigned long long), st));
    for (int mode = 0; mode < 2; ++mode) {
        BSW_TRY(launch_mate_prepare(d_pairs, d_aln, n, mode, s.d_mmeta, s.d_mjobs, (int32_t)jcap, st));
        BSW_TRY(hipMemcpyAsync(s.h_mmeta, s.d_mmeta, kMateMetaWords * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        BSW_TRY(hipStreamSynchronize(st));
        const int32_t *m = s.h_mmeta;
        if (m[kMateMetaErr]) return BSW_E_RANGE;
        int32_t njobs = 0;
        for (int b = 0; b < kMateBuckets; ++b) njobs += m[kMateMetaCount + b];
        const int64_t total = m[kMateMetaTotal];
        uint16_t *rows = nullptr;
        if (mode == 0 && njobs > 0) {
            const size_t need = (size_t)std::max(m[kMateMetaTmax], 1) * (size_t)total;
            BSW_TRY(grow(s.d_mrows, s.cap_mrows, need));
            rows = s.d_mrows;
        }
        hipEvent_t e0 = mode == 0 ? s.ev0 : s.ev2, e1 = mode == 0 ? s.ev1 : s.ev3;
        BSW_TRY(hipEventRecord(e0, st));
        for (int c = 0; c < kMateClasses; ++c)
            BSW_TRY(launch_mate_class(c, mp, d_pairs, s.d_mjobs, m[kMateMetaClass + 2 * c],
                                      m[kMateMetaClass + 2 * c + 1], d_ref, d_qer, d_aln, mode, rows, total,
                                      mode == 0 ? s.d_mcells : nullptr, st));
        BSW_TRY(hipEventRecord(e1, st));
        if (mode == 0) stats->n_fwd = njobs; else stats->n_rev = njobs;
    }
    unsigned long long cells = 0;
    BSW_TRY(hipMemcpyAsync(&cells, s.d_mcells, sizeof(cells), hipMemcpyDeviceToHost, st));
    BSW_TRY(hipStreamSynchronize(st));
    BSW_TRY(hipEventElapsedTime(&stats->fwd_ms, s.ev0, s.ev1));
    BSW_TRY(hipEventElapsedTime(&stats->rev_ms, s.ev2, s.ev3));
    stats->cells_fwd = (int64_t)cells;
    return BSW_OK;
}

// ---------------------------------------------------------------- global alignment (bsw_global.h)
static void make_glob_params(const bsw_params_t &p, int prefer_band, GlobParams &gp)
{
    memset(&gp, 0, sizeof(gp));
    gp.o_del = p.o_del; gp.e_del = p.e_del; gp.o_ins = p.o_ins; gp.e_ins = p.e_ins;
    gp.oe_del = p.o_del + p.e_del; gp.oe_ins = p.o_ins + p.e_ins;
    int mx = 0;
    for (int i = 0; i < 25; ++i) mx = std::max(mx, std::abs((int)p.mat[i]));
    gp.maxabs = mx;
    memcpy(gp.mat, p.mat, 25);
    gp.prefer_band = prefer_band ? 1 : 0;
    for (int t = 0; t < 8; ++t) {                        // codes > 4 score as N (as prof in KParams)
        const int tt = std::min(t, 4);
        uint8_t b[8];
        for (int q = 0; q < 8; ++q) b[q] = (uint8_t)p.mat[tt * 5 + std::min(q, 4)];
        gp.prof[t][0] = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
        gp.prof[t][1] = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
    }
}

constexpr int64_t kGlobZCapWords = (int64_t)2 << 30;     // traceback matrix per launch <= 8 GB

// plan -> sort (class, w, qlen, tlen) -> one readback of the class statistics -> per class the
// DP + traceback kernel over its slice of order[] (chunked so the matrix stays under the cap).
static int glob_device(const GlobParams &gp, Slot &s, SeqPair *d_pairs, const uint8_t *d_ref,
                       const uint8_t *d_qer, int32_t n, uint32_t *d_cigar, int32_t stride, int32_t *d_ncig,
                       hipStream_t st, bsw_global_stats_t *stats)
{
    *stats = bsw_global_stats_t{};
    stats->n_jobs = n;
    if (n == 0) return BSW_OK;
    BSW_TRY(grow_sort(s, n));
    if (!s.d_gmeta) BSW_TRY(hipMalloc((void **)&s.d_gmeta, kGMetaWords * sizeof(int32_t)));
    if (!s.h_gmeta) BSW_TRY(hipHostMalloc((void **)&s.h_gmeta, kGMetaWords * sizeof(int32_t), 0));
    if (!s.d_mcells) BSW_TRY(hipMalloc((void **)&s.d_mcells, sizeof(unsigned long long)));
    BSW_TRY(launch_glob_plan(d_pairs, n, gp, s.d_keys, s.d_vals, s.d_gmeta, st));
    size_t tmp_bytes = 0;
    BSW_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, s.d_keys, s.d_keys2, s.d_vals, s.d_order, n,
                                               0, kGlobKeyBits, st));
    BSW_TRY(grow(s.d_tmp, s.cap_tmp, tmp_bytes));
    BSW_TRY(hipcub::DeviceRadixSort::SortPairs(s.d_tmp, tmp_bytes, s.d_keys, s.d_keys2, s.d_vals, s.d_order, n,
                                               0, kGlobKeyBits, st));
    BSW_TRY(hipMemcpyAsync(s.h_gmeta, s.d_gmeta, kGMetaWords * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    BSW_TRY(hipMemsetAsync(s.d_mcells, 0, sizeof(unsigned long long), st));
    BSW_TRY(hipStreamSynchronize(st));
    int32_t m[kGMetaWordsPerSlot] = {};
    for (int sl = 0; sl < kGMetaSpread; ++sl) {
        const int32_t *v = s.h_gmeta + sl * kGMetaWordsPerSlot;
        for (int c = 0; c < kGlobClasses; ++c) {
            m[kGMetaCount + c] += v[kGMetaCount + c];
            m[kGMetaTmax + c] = std::max(m[kGMetaTmax + c], v[kGMetaTmax + c]);
            m[kGMetaWmax + c] = std::max(m[kGMetaWmax + c], v[kGMetaWmax + c]);
            m[kGMetaQmax + c] = std::max(m[kGMetaQmax + c], v[kGMetaQmax + c]);
        }
        m[kGMetaErr] |= v[kGMetaErr];
    }
    if (m[kGMetaErr]) return BSW_E_RANGE;
    const bool want = d_cigar && stride > 0;
    // column classes keep only a narrow corridor of the traceback matrix (glob_lane_kernel: 3 dwords
    // per row instead of the band's ~10 at bwa-shaped w); jobs whose path leaves it rerun below with
    // the full band window
    constexpr int tb_env = 3;
    if (want) BSW_TRY(grow(s.d_gretry, s.cap_gretry, (size_t)n + 1));
    BSW_TRY(hipEventRecord(s.ev0, st));
    int32_t off = 0;
    for (int c = 0; c < kGlobClasses; ++c) {
        const int32_t cnt = m[kGMetaCount + c];
        if (cnt <= 0) continue;
        const int tm = m[kGMetaTmax + c], wm = m[kGMetaWmax + c], qm = m[kGMetaQmax + c];
        const int cap_dw = glob_cap_dw(c, qm, wm);
        const bool col = c >= kGlobLane0 && c < kGlobWideClass;
        const int tb = (want && col && tb_env > 0 && tb_env < cap_dw) ? tb_env : 0;
        // one pass over the class (narrow window when tb > 0), then the retry list with the full window
        for (int pass = 0; pass < (tb > 0 ? 2 : 1); ++pass) {
            const int ptb = pass == 0 ? tb : 0;
            int32_t pcnt = cnt;
            const int32_t *ord = s.d_order + off;
            if (pass == 1) {                                // the jobs the narrow window could not serve
                int32_t nr = 0;
                BSW_TRY(hipMemcpyAsync(&nr, s.d_gretry, sizeof(int32_t), hipMemcpyDeviceToHost, st));
                BSW_TRY(hipStreamSynchronize(st));
                stats->n_tb_retry += nr;
                if (nr <= 0) break;
                pcnt = nr;
                ord = s.d_gretry + 1;
            } else if (ptb > 0) {
                BSW_TRY(hipMemsetAsync(s.d_gretry, 0, sizeof(int32_t), st));
            }
            const int64_t zstride = (int64_t)std::max(tm, 1) * (ptb > 0 ? ptb : cap_dw) * 64;
            int32_t chunk = pcnt;
            if (want) {
                const int64_t waves = std::max<int64_t>(1, kGlobZCapWords / zstride);
                chunk = (int32_t)std::min<int64_t>(pcnt, waves * 64);
                BSW_TRY(grow(s.d_gz, s.cap_gz, (size_t)((chunk + 63) / 64) * (size_t)zstride));
            }
            if (c == kGlobWideClass) BSW_TRY(grow(s.d_scratch, s.cap_scratch, (size_t)(qm + 1) * (size_t)chunk));
            for (int32_t a = 0; a < pcnt; a += chunk) {
                const int32_t b = std::min(pcnt, a + chunk);
                BSW_TRY(launch_glob_class(c, gp, d_pairs, ord + a, b - a, d_ref, d_qer,
                                          want ? s.d_gz : nullptr, zstride, cap_dw, s.d_scratch, d_cigar, stride,
                                          d_ncig, pass == 0 ? s.d_mcells : nullptr, st, ptb,
                                          ptb > 0 ? s.d_gretry : nullptr));
                stats->n_launches++;
                if (want) stats->z_bytes += (int64_t)((b - a + 63) / 64) * zstride * 4;
            }
        }
        if (c == kGlobWideClass) stats->n_wide += cnt;
        else stats->n_lane += cnt;
        off += cnt;
    }
    BSW_TRY(hipEventRecord(s.ev1, st));
    unsigned long long cells = 0;
    BSW_TRY(hipMemcpyAsync(&cells, s.d_mcells, sizeof(cells), hipMemcpyDeviceToHost, st));
    BSW_TRY(hipStreamSynchronize(st));
    BSW_TRY(hipEventElapsedTime(&stats->kernel_ms, s.ev0, s.ev1));
    stats->cells = (int64_t)cells;
    return BSW_OK;
}

// ---------------------------------------------------------------- device extension pipeline
// One side of bsw_extend_seeds on the GPU: build (sparse job per read) -> engine -> band retries
// -> interpretation.  Every step on `st`; the only host syncs are the engine's class-count
// readback and one retry count per retry round.
static int ext_side_device(const KParams &kp0, Slot &s, const ExtDevParams &xp, int left, const bsw_ext_opt_t &opt,
                           const uint8_t *d_reads, const int64_t *d_off, const int32_t *d_len,
                           const bsw_seed_t *d_seeds, const int64_t *d_win, int32_t n, const uint8_t *d_ref,
                           bsw_alnreg_t *d_out, int32_t *d_cnt, hipStream_t st, bsw_ext_stats_t &es)
{
    KParams kp = kp0;
    kp.end_bonus = left ? opt.pen_clip5 : opt.pen_clip3;
    BSW_TRY(launch_ext_build(left, xp, d_reads, d_off, d_len, d_seeds, d_win, n, d_ref, s.d_xst, s.d_xpairs, s.d_xq,
                             s.d_xt, d_out, st));
    int r = run_device(kp, s, s.d_xpairs, s.d_xt, s.d_xq, n, opt.w, 16, st);
    if (r) return r;
    // each DP batch, the next band-retry mark and its count readback are queued before one wait
    // (finish_stats), so a retry level costs one host round trip, not two
    for (int t = 1;; ++t) {
        const bool retry = t < opt.max_band_try;
        const int32_t wt = opt.w << (t - 1), wn = opt.w << t;
        if (retry) {
            BSW_TRY(launch_ext_retry_mark(t == 1 ? s.d_xpairs : s.d_xsub, s.d_xsub, s.d_xst, n, wt, d_cnt, st));
            BSW_TRY(hipMemcpyAsync(s.h_meta + kMetaCnt, d_cnt, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        }
        if ((r = finish_stats(s))) return r;
        es.kernel_ms += s.stats.kernel_ms;
        if (!retry) break;
        BSW_TRY(hipStreamSynchronize(st));          // (idle already unless the batch was empty)
        const int32_t cnt = s.h_meta[kMetaCnt];
        if (cnt == 0) break;
        es.n_pairs[(left ? 0 : 2) + 1] += cnt;
        if ((r = run_device(kp, s, s.d_xsub, s.d_xt, s.d_xq, n, wn, 16, st))) return r;
        BSW_TRY(launch_ext_retry_merge(s.d_xpairs, s.d_xsub, s.d_xst, n, wn, left, st));
    }
    BSW_TRY(launch_ext_interp(left, xp, d_len, d_seeds, n, s.d_xpairs, s.d_xst, d_out, st));
    return BSW_OK;
}

}  // namespace bsw

// ====================================================================== C ABI
extern "C" {

void bsw_params_default(bsw_params_t *p)
{
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->o_del = p->o_ins = 6;
    p->e_del = p->e_ins = 1;
    p->zdrop = 100;
    p->end_bonus = 5;
    p->w_match = 1;
    p->w_mismatch = -4;
    p->w_ambig = -1;
    for (int t = 0; t < 5; ++t)
        for (int q = 0; q < 5; ++q)
            p->mat[t * 5 + q] = (t == 4 || q == 4) ? -1 : (t == q ? 1 : -4);
}

static bool params_ok(const bsw_params_t *p)
{
    if (p->e_del < 1 || p->e_ins < 1 || p->o_del < 0 || p->o_ins < 0) return false;
    if (p->o_del + p->e_del > 32767 || p->o_ins + p->e_ins > 32767) return false;
    return true;
}

int bsw_create_on(const bsw_params_t *params, const int *devices, int n_devices, bsw_ctx_t **out)
{
    if (!params || !out || !devices || n_devices < 1 || !params_ok(params)) return BSW_E_INVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return BSW_E_NODEV;
    for (int d = 0; d < n_devices; ++d)
        if (devices[d] < 0 || devices[d] >= ndev) return BSW_E_NODEV;
    auto *c = new bsw_ctx();
    c->params = *params;
    bsw::make_kparams(*params, c->kp);
    for (int d = 0; d < n_devices; ++d) {
        auto dc = std::make_unique<bsw::DeviceCtx>();
        dc->device = devices[d];
        c->devs.push_back(std::move(dc));
    }
    *out = c;
    return BSW_OK;
}

int bsw_create(const bsw_params_t *params, int device0, int n_gpus, bsw_ctx_t **out)
{
    if (!params || !out || n_gpus < 1 || device0 < 0 || n_gpus > 4096) return BSW_E_INVAL;
    std::vector<int> devs((size_t)n_gpus);
    for (int d = 0; d < n_gpus; ++d) devs[d] = device0 + d;
    return bsw_create_on(params, devs.data(), n_gpus, out);
}

void bsw_destroy(bsw_ctx_t *ctx) { delete ctx; }

static int validate(const SeqPair *pairs, int32_t n, int32_t w, int cell_bits)
{
    if (n < 0 || w < 0 || (cell_bits != 8 && cell_bits != 16)) return BSW_E_INVAL;
    if (n > 0 && !pairs) return BSW_E_INVAL;
    return BSW_OK;
}

}  // extern "C"

namespace bsw {

// Static band cells of one pair (rows i < tlen, columns [max(0, i - w), min(qlen, i + w + 1))):
// the work estimate behind the multi-device split.
static int64_t band_cells_est(int64_t qlen, int64_t tlen, int64_t w)
{
    if (qlen <= 0 || tlen <= 0) return 0;
    const int64_t T = std::min(tlen, qlen + w);                  // rows with a non-empty band
    auto ssum = [](int64_t a, int64_t b, int64_t c) {            // sum_{i=a}^{b-1} (i + c)
        return b > a ? (b - a) * (a + b - 1) / 2 + c * (b - a) : (int64_t)0;
    };
    const int64_t k = std::min(T, std::max<int64_t>(qlen - w, 0));   // rows with i + w + 1 <= qlen
    const int64_t hi = ssum(0, k, w + 1) + qlen * (T - k);
    const int64_t lo = ssum(std::min(T, w + 1), T, -w);              // rows with i > w
    return std::max<int64_t>(hi - lo, 0);
}

// nd + 1 cut points: device d takes pairs [cut[d], cut[d+1]), each range ~1/nd of the cells
// (plus a per-pair constant for the plan / sort / launch share)
static std::vector<int32_t> split_by_cells(const SeqPair *pairs, int32_t n, int32_t w, int nd)
{
    std::vector<int64_t> pre((size_t)n + 1, 0);
    for (int32_t i = 0; i < n; ++i)
        pre[i + 1] = pre[i] + 64 + band_cells_est(pairs[i].len2, pairs[i].len1, w);
    std::vector<int32_t> cut((size_t)nd + 1, n);
    cut[0] = 0;
    for (int d = 1; d < nd; ++d) {
        const int64_t target = pre[n] * d / nd;
        cut[d] = (int32_t)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
        cut[d] = std::max(cut[d], cut[d - 1]);
    }
    return cut;
}

// Multi-device policy (a context over several logical devices): a call of fewer than
// split_min items runs whole on ONE device -- the one with the fewest host-buffer calls in
// flight, ties rotating -- so kt_for-sized calls from concurrent workers spread over the
// devices instead of each paying every device's launch latency for a sliver of work; larger
// calls split into contiguous ranges, one per device.  Returns the device, or -1: split.
struct Inflight {
    DeviceCtx &dc;
    explicit Inflight(DeviceCtx &d) : dc(d) { dc.inflight.fetch_add(1); }
    ~Inflight() { dc.inflight.fetch_sub(1); }
};

static int one_device(bsw_ctx_t *ctx, int64_t n)
{
    const int nd = (int)ctx->devs.size();
    if (nd == 1) return 0;
    if (n >= ctx->split_min) return -1;
    const unsigned r = ctx->rr.fetch_add(1);
    int best = -1, load = INT32_MAX;
    for (int k = 0; k < nd; ++k) {
        const int d = (int)((r + (unsigned)k) % (unsigned)nd);
        const int l = ctx->devs[d]->inflight.load();
        if (l < load) { load = l; best = d; }
    }
    return best;
}

// Recovery of a host-buffer range whose run on device d0 failed with BSW_E_NOMEM / BSW_E_HIP
// (bsw.h, bsw_get_scores): 1. again on d0 after its cached slots are freed, 2. on each other
// device of the context, 3. (BSW_E_NOMEM only) in halves (down to one 4096-pair staging block),
// each half the same way.  No coalescing here: the range runs as a call of its own.  Outputs are identical to an
// undisturbed call -- pairs are independent, and a failed run writes no input field (staged
// records go back as outputs only or as the caller's own bytes).  `how` gets the deepest step
// used.  Upstream plans to degrade on engine errors instead of aborting the run
// (PHASE2_IMPLEMENTATION_SUMMARY.md:210-225); there is no CPU path to degrade to here.
static bool recoverable(int rc) { return rc == BSW_E_NOMEM || rc == BSW_E_HIP; }

static int recover_range(bsw_ctx_t *ctx, const KParams &kp, int d0, SeqPair *pairs, const uint8_t *ref,
                         const uint8_t *qer, int32_t n, int32_t w, int cell_bits, bsw_stats_t *st, int &how)
{
    const int nd = (int)ctx->devs.size();
    int rc = BSW_E_HIP;
    for (int k = 0; k < nd; ++k) {
        const int d = (d0 + k) % nd;
        DeviceCtx &dc = *ctx->devs[d];
        dc.trim();
        {
            Inflight g(dc);
            rc = host_shard(kp, dc, pairs, ref, qer, n, w, cell_bits, ctx->host_chunk, ctx->host_pack == 2, st);
        }
        if (rc == BSW_OK) {
            how = std::max(how, k == 0 ? 1 : 2);
            return BSW_OK;
        }
        if (!recoverable(rc)) return rc;
    }
    // halves only for memory: a smaller range needs smaller buffers, but it cannot fix a HIP error
    // (a sticky context error repeats on every rerun)
    if (rc != BSW_E_NOMEM || n <= kStageBlk) return rc;
    const int32_t h = std::max<int32_t>(kStageBlk, (n / 2) & ~(kStageBlk - 1));
    bsw_stats_t a{}, b{};
    if ((rc = recover_range(ctx, kp, d0, pairs, ref, qer, h, w, cell_bits, &a, how))) return rc;
    if ((rc = recover_range(ctx, kp, (d0 + 1) % nd, pairs + h, ref, qer, n - h, w, cell_bits, &b, how))) return rc;
    how = std::max(how, 3);
    *st = a;
    st->kernel_ms += b.kernel_ms; st->stage_ms += b.stage_ms; st->host_ms += b.host_ms;
    st->n_i16 += b.n_i16; st->n_u8 += b.n_u8; st->n_wide += b.n_wide; st->n_packed += b.n_packed;
    st->n_launches += b.n_launches; st->n_wave += b.n_wave; st->n_group += b.n_group;
    return BSW_OK;
}

int scores_eb(bsw_ctx_t *ctx, int32_t end_bonus, SeqPair *pairs, const uint8_t *seqBufRef,
              const uint8_t *seqBufQer, int32_t n, int32_t w, int cell_bits, bsw_stats_t *out)
{
    if (!ctx) return BSW_E_INVAL;
    int rc = validate(pairs, n, w, cell_bits);
    if (rc) return rc;
    *out = bsw_stats_t{};
    if (n == 0) return BSW_OK;
    if (!seqBufRef || !seqBufQer) return BSW_E_INVAL;
    KParams kp = ctx->kp;
    kp.end_bonus = end_bonus;
    const int one = one_device(ctx, n);
    const int nd = one >= 0 ? 1 : (int)ctx->devs.size();
    // one device: host_shard's parallel pre-pass validates; several: validate the whole batch
    // before any device starts
    if (nd > 1)
        for (int32_t i = 0; i < n; ++i)
            if (pairs[i].len1 < 0 || pairs[i].len2 < 0 || pairs[i].len1 > BSW_MAX_LEN ||
                pairs[i].len2 > BSW_MAX_LEN || pairs[i].idr < 0 || pairs[i].idq < 0)
                return BSW_E_RANGE;
    std::vector<int> rcs(nd, BSW_OK);
    std::vector<bsw_stats_t> st(nd);
    std::vector<int> how(nd, 0);
    if (nd == 1) {
        {
            Inflight g(*ctx->devs[one]);
            if (n <= ctx->coalesce)             // kt_for-sized: coalesce with concurrent callers
                rcs[0] = coalesced_call(kp, *ctx->devs[one], pairs, seqBufRef, seqBufQer, n, w, cell_bits,
                                        ctx->host_chunk, ctx->host_pack == 2, &st[0]);
            else
                rcs[0] = host_shard(kp, *ctx->devs[one], pairs, seqBufRef, seqBufQer, n, w, cell_bits,
                                    ctx->host_chunk, ctx->host_pack == 2, &st[0]);
        }
        if (recoverable(rcs[0]))
            rcs[0] = recover_range(ctx, kp, one, pairs, seqBufRef, seqBufQer, n, w, cell_bits, &st[0], how[0]);
    } else {
        // contiguous pair ranges of equal estimated work (static band cells)
        const std::vector<int32_t> cut = split_by_cells(pairs, n, w, nd);
        std::vector<std::thread> th;
        for (int d = 0; d < nd; ++d) {
            const int32_t a = cut[d], b = cut[d + 1];
            th.emplace_back([&, d, a, b] {
                {
                    Inflight g(*ctx->devs[d]);
                    rcs[d] = host_shard(kp, *ctx->devs[d], pairs + a, seqBufRef, seqBufQer, b - a, w,
                                        cell_bits, ctx->host_chunk, ctx->host_pack == 2, &st[d]);
                }
                if (recoverable(rcs[d]))
                    rcs[d] = recover_range(ctx, kp, d, pairs + a, seqBufRef, seqBufQer, b - a, w, cell_bits, &st[d],
                                           how[d]);
            });
        }
        for (auto &t : th) t.join();
    }
    bsw_stats_t agg{};
    for (int d = 0; d < nd; ++d) {
        if (rcs[d]) return rcs[d];
        agg.kernel_ms = std::max(agg.kernel_ms, st[d].kernel_ms);
        agg.n_i16 += st[d].n_i16; agg.n_u8 += st[d].n_u8; agg.n_wide += st[d].n_wide; agg.n_packed += st[d].n_packed;
        agg.n_launches += st[d].n_launches;
        agg.n_wave += st[d].n_wave; agg.n_group += st[d].n_group;
        agg.stage_ms = std::max(agg.stage_ms, st[d].stage_ms);
        agg.host_ms = std::max(agg.host_ms, st[d].host_ms);
        agg.recovery = std::max(agg.recovery, how[d]);
    }
    agg.n_devices = nd;
    *out = agg;
    return BSW_OK;
}

void ctx_params(const bsw_ctx_t *ctx, bsw_params_t *out) { *out = ctx->params; }
int ctx_device(const bsw_ctx_t *ctx) { return ctx->devs[0]->device; }
int64_t ctx_refres_len(bsw_ctx_t *ctx)
{
    bsw::DeviceCtx &dc = *ctx->devs[0];
    std::shared_lock<std::shared_mutex> g(dc.refmu);
    return dc.d_refres ? dc.refres_len : -1;
}

void *pinned_acquire(bsw_ctx_t *ctx, int which, size_t bytes)
{
    auto &b = ctx->pin[which & 1];
    if (!b.mu.try_lock()) return nullptr;
    if (b.cap < bytes) {
        if (b.p) (void)hipHostFree(b.p);
        b.p = nullptr; b.cap = 0;
        const size_t cap = std::max(bytes, b.cap + b.cap / 2);
        if (hipHostMalloc(&b.p, cap, 0) != hipSuccess) { b.p = nullptr; b.mu.unlock(); return nullptr; }
        b.cap = cap;
    }
    return b.p;
}

void pinned_release(bsw_ctx_t *ctx, int which) { ctx->pin[which & 1].mu.unlock(); }

// reads per extension call chunk: the int32-offset bound, optionally lowered per context
// (BSW_OPT_EXT_CHUNK: exercises the chunked paths at small sizes)
int64_t ext_chunk_cap(const bsw_ctx_t *ctx)
{
    return ctx->ext_chunk > 0 ? ctx->ext_chunk : (int64_t)INT32_MAX;
}

void set_chain_stats(bsw_ctx_t *ctx, const bsw_chain_stats_t &s)
{
    std::lock_guard<std::mutex> g(ctx->stats_mu);
    ctx->chain_last = s;
}

int get_chain_stats(bsw_ctx_t *ctx, bsw_chain_stats_t *out)
{
    if (!ctx || !out) return BSW_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->stats_mu);
    *out = ctx->chain_last;
    return BSW_OK;
}

void set_ext_stats(bsw_ctx_t *ctx, const bsw_ext_stats_t &s)
{
    std::lock_guard<std::mutex> g(ctx->stats_mu);
    ctx->ext_last = s;
}

int get_ext_stats(bsw_ctx_t *ctx, bsw_ext_stats_t *out)
{
    if (!ctx || !out) return BSW_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->stats_mu);
    *out = ctx->ext_last;
    return BSW_OK;
}

}  // namespace bsw

extern "C" {

int bsw_get_scores(bsw_ctx_t *ctx, SeqPair *pairs, const uint8_t *seqBufRef,
                   const uint8_t *seqBufQer, int32_t n, int32_t w, int cell_bits)
{
    if (!ctx) return BSW_E_INVAL;
    bsw_stats_t st{};
    const int rc = bsw::scores_eb(ctx, ctx->params.end_bonus, pairs, seqBufRef, seqBufQer, n, w,
                                  cell_bits, &st);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(ctx->stats_mu);
    ctx->last = st;
    return BSW_OK;
}

int bsw_get_scores_device(bsw_ctx_t *ctx, SeqPair *d_pairs, const uint8_t *d_ref,
                          const uint8_t *d_qer, int32_t n, int32_t w, int cell_bits, void *stream)
{
    if (!ctx) return BSW_E_INVAL;
    int rc = validate(d_pairs, n, w, cell_bits);
    if (rc) return rc;
    if (n == 0) return BSW_OK;
    if (!d_ref || !d_qer) return BSW_E_INVAL;
    bsw::DeviceCtx &dc = *ctx->devs[0];
    auto slot = dc.acquire(rc);
    if (!slot) return rc;
    rc = [&]() -> int {
        BSW_TRY(hipSetDevice(dc.device));
        hipStream_t st = stream ? (hipStream_t)stream : slot->stream;
        int r = bsw::run_device(ctx->kp, *slot, d_pairs, d_ref, d_qer, n, w, cell_bits, st);
        if (r) return r;
        if ((r = bsw::finish_stats(*slot))) return r;
        std::lock_guard<std::mutex> g(ctx->stats_mu);
        ctx->last = slot->stats;
        return BSW_OK;
    }();
    dc.give_back(std::move(slot), rc);
    return rc;
}

// The packed wire form (bsw_pack_batch) scored in place: one stage_in_kernel (2-bit unpack of both
// extents, exception patches, 20-B records -> SeqPair, pads zeroed), the device pipeline, then the
// 24 output bytes per pair compacted into d_out -- the path of a batch that arrived over RCCL
int bsw_get_scores_packed_device(bsw_ctx_t *ctx, const void *d_packed, const bsw_packed_t *desc, int32_t w,
                                 int cell_bits, int32_t *d_out, void *stream)
{
    if (!ctx || !desc) return BSW_E_INVAL;
    const bsw_packed_t d = *desc;
    if (d.n < 0 || w < 0 || (cell_bits != 8 && cell_bits != 16)) return BSW_E_INVAL;
    if (d.n == 0) return BSW_OK;
    if (!d_packed || !d_out || d.ref_bytes < 0 || d.qer_bytes < 0 || d.n_exc_ref < 0 || d.n_exc_qer < 0 ||
        d.ref_bytes >= ((int64_t)1 << 30) || d.qer_bytes >= ((int64_t)1 << 30) ||
        ((d.rec_off | d.ref_off | d.qer_off | d.exc_off) & 3) != 0)
        return BSW_E_INVAL;
    bsw::DeviceCtx &dc = *ctx->devs[0];
    int rc = BSW_OK;
    auto slot = dc.acquire(rc);
    if (!slot) return rc;
    bsw::Slot &s = *slot;
    rc = [&]() -> int {
        BSW_TRY(hipSetDevice(dc.device));
        hipStream_t st = stream ? (hipStream_t)stream : s.stream;
        BSW_TRY(bsw::grow(s.d_ref, s.cap_ref, (size_t)d.ref_bytes + 16));
        BSW_TRY(bsw::grow(s.d_qer, s.cap_qer, (size_t)d.qer_bytes + 16));
        BSW_TRY(bsw::grow(s.d_pairs, s.cap_pairs, (size_t)d.n));
        const uint8_t *b = (const uint8_t *)d_packed;
        // the staging kernels on the slot's high-priority stream (after the caller's stream: the
        // piece may have been written there), as plan / sort already are: a piece's preparation is
        // then dispatched ahead of another piece's queued DP workgroups instead of behind them (the
        // RCCL leg's trace: the second piece's staging waited out the first piece's whole DP,
        // profiles/r06/rccl_leg_trace.txt).  Its DP, on `st`, waits for the plan (run_dp).
        if (int e = bsw::ensure_pstream(s)) return e;
        BSW_TRY(hipEventRecord(s.evh, st));
        BSW_TRY(hipStreamWaitEvent(s.pstream, s.evh, 0));
        if (int e = bsw::launch_stage_in(s, s.pstream, b + d.ref_off, d.ref_bytes, b + d.qer_off, d.qer_bytes,
                                         (const uint32_t *)(b + d.exc_off), d.n_exc_ref, d.n_exc_ref + d.n_exc_qer,
                                         (const bsw::PairIn *)(b + d.rec_off), d.n, s.d_ref, s.d_qer, s.d_pairs, nullptr))
            return e;
        // everything after it on `st` (the small-batch route launches there without a plan)
        BSW_TRY(hipEventRecord(s.evh, s.pstream));
        BSW_TRY(hipStreamWaitEvent(st, s.evh, 0));
        int r = bsw::run_device(ctx->kp, s, s.d_pairs, s.d_ref, s.d_qer, d.n, w, cell_bits, st);
        if (r) return r;
        if ((r = bsw::finish_stats(s))) return r;
        hipLaunchKernelGGL(bsw::gather_outputs_kernel, dim3((unsigned)((d.n + 255) / 256)), dim3(256), 0, st,
                           s.d_pairs, d_out, d.n);
        BSW_TRY(hipGetLastError());
        BSW_TRY(hipStreamSynchronize(st));
        std::lock_guard<std::mutex> g(ctx->stats_mu);
        ctx->last = s.stats;
        return BSW_OK;
    }();
    dc.give_back(std::move(slot), rc);
    return rc;
}

int bsw_ksw_align2_device(bsw_ctx_t *ctx, const SeqPair *d_pairs, const uint8_t *d_ref,
                          const uint8_t *d_qer, int32_t n, bsw_kswr_t *d_aln, void *stream)
{
    if (!ctx || n < 0 || (n > 0 && (!d_pairs || !d_ref || !d_qer || !d_aln))) return BSW_E_INVAL;
    if (!bsw::mate_params_ok(ctx->params)) return BSW_E_INVAL;
    if (n == 0) return BSW_OK;
    bsw::MateParams mp;
    bsw::make_mate_params(ctx->params, mp);
    bsw::DeviceCtx &dc = *ctx->devs[0];
    int rc = BSW_OK;
    auto slot = dc.acquire(rc);
    if (!slot) return rc;
    rc = [&]() -> int {
        BSW_TRY(hipSetDevice(dc.device));
        hipStream_t st = stream ? (hipStream_t)stream : slot->stream;
        bsw_mate_stats_t ms;
        const int r = bsw::mate_device(mp, *slot, d_pairs, d_ref, d_qer, n, d_aln, st, &ms);
        if (r) return r;
        std::lock_guard<std::mutex> g(ctx->stats_mu);
        ctx->mate_last = ms;
        return BSW_OK;
    }();
    dc.give_back(std::move(slot), rc);
    return rc;
}

}  // extern "C"

namespace bsw {
// One device's share of a host-buffer mate-rescue call (contiguous job range).
static int mate_host_shard(const MateParams &mp, DeviceCtx &dc, const SeqPair *pairs, const uint8_t *seqBufRef,
                           const uint8_t *seqBufQer, int32_t n, bsw_kswr_t *aln, bsw_mate_stats_t *ms)
{
    *ms = bsw_mate_stats_t{};
    if (n == 0) return BSW_OK;
    int rc = BSW_OK;
    auto slot = dc.acquire(rc);
    if (!slot) return rc;
    Slot &s = *slot;
    rc = [&]() -> int {
        BSW_TRY(hipSetDevice(dc.device));
        int64_t r_lo = INT64_MAX, r_hi = 0, q_lo = INT64_MAX, q_hi = 0;
        for (int32_t i = 0; i < n; ++i) {
            const SeqPair &p = pairs[i];
            if (p.len1 > 0) { r_lo = std::min<int64_t>(r_lo, p.idr); r_hi = std::max<int64_t>(r_hi, (int64_t)p.idr + p.len1); }
            if (p.len2 > 0) { q_lo = std::min<int64_t>(q_lo, p.idq); q_hi = std::max<int64_t>(q_hi, (int64_t)p.idq + p.len2); }
        }
        if (r_lo == INT64_MAX) r_lo = r_hi = 0;
        if (q_lo == INT64_MAX) q_lo = q_hi = 0;
        BSW_TRY(grow(s.d_mpairs, s.cap_mpairs, (size_t)n));
        BSW_TRY(grow(s.d_maln, s.cap_maln, (size_t)n));
        BSW_TRY(grow(s.d_ref, s.cap_ref, (size_t)(r_hi - r_lo) + 1));
        BSW_TRY(grow(s.d_qer, s.cap_qer, (size_t)(q_hi - q_lo) + 1));
        BSW_TRY(hipMemcpyAsync(s.d_mpairs, pairs, (size_t)n * sizeof(SeqPair), hipMemcpyHostToDevice, s.stream));
        if (r_hi > r_lo) BSW_TRY(hipMemcpyAsync(s.d_ref, seqBufRef + r_lo, (size_t)(r_hi - r_lo), hipMemcpyHostToDevice, s.stream));
        if (q_hi > q_lo) BSW_TRY(hipMemcpyAsync(s.d_qer, seqBufQer + q_lo, (size_t)(q_hi - q_lo), hipMemcpyHostToDevice, s.stream));
        int r = mate_device(mp, s, s.d_mpairs, s.d_ref - r_lo, s.d_qer - q_lo, n, s.d_maln, s.stream, ms);
        if (r) return r;
        BSW_TRY(hipMemcpyAsync(aln, s.d_maln, (size_t)n * sizeof(bsw_kswr_t), hipMemcpyDeviceToHost, s.stream));
        BSW_TRY(hipStreamSynchronize(s.stream));
        return BSW_OK;
    }();
    dc.give_back(std::move(slot), rc);
    return rc;
}

// Run shard(d, a, b) for contiguous job ranges [a, b) on every device of the context (one host
// thread per device; jobs are independent), first non-zero status wins.
// Small calls run whole on one device (one_device's policy).
template <class F>
static int shard_devices(bsw_ctx_t *ctx, int32_t n, F shard)
{
    const int one = one_device(ctx, n);
    if (one >= 0) {
        Inflight g(*ctx->devs[one]);
        return shard(one, 0, n);
    }
    const int nd = (int)ctx->devs.size();
    std::vector<int> rcs(nd, BSW_OK);
    std::vector<std::thread> th;
    for (int d = 0; d < nd; ++d) {
        const int32_t a = (int32_t)((int64_t)n * d / nd), b = (int32_t)((int64_t)n * (d + 1) / nd);
        th.emplace_back([&, d, a, b] {
            Inflight g(*ctx->devs[d]);
            rcs[d] = shard(d, a, b);
        });
    }
    for (auto &t : th) t.join();
    for (int r : rcs)
        if (r) return r;
    return BSW_OK;
}
}  // namespace bsw

extern "C" {

int bsw_ksw_align2(bsw_ctx_t *ctx, const SeqPair *pairs, const uint8_t *seqBufRef, const uint8_t *seqBufQer,
                   int32_t n, bsw_kswr_t *aln)
{
    if (!ctx || n < 0 || (n > 0 && (!pairs || !seqBufRef || !seqBufQer || !aln))) return BSW_E_INVAL;
    if (!bsw::mate_params_ok(ctx->params)) return BSW_E_INVAL;
    if (n == 0) return BSW_OK;
    for (int32_t i = 0; i < n; ++i)
        if (pairs[i].len1 < 0 || pairs[i].len2 < 0 || pairs[i].len1 > BSW_MAX_LEN ||
            pairs[i].len2 > BSW_MATE_MAX_QLEN || pairs[i].idr < 0 || pairs[i].idq < 0)
            return BSW_E_RANGE;
    bsw::MateParams mp;
    bsw::make_mate_params(ctx->params, mp);
    std::vector<bsw_mate_stats_t> st(ctx->devs.size());
    const int rc = bsw::shard_devices(ctx, n, [&](int d, int32_t a, int32_t b) {
        return bsw::mate_host_shard(mp, *ctx->devs[d], pairs + a, seqBufRef, seqBufQer, b - a, aln + a, &st[d]);
    });
    if (rc) return rc;
    bsw_mate_stats_t agg{};
    for (const auto &x : st) {
        agg.fwd_ms = std::max(agg.fwd_ms, x.fwd_ms); agg.rev_ms = std::max(agg.rev_ms, x.rev_ms);
        agg.n_fwd += x.n_fwd; agg.n_rev += x.n_rev; agg.cells_fwd += x.cells_fwd;
    }
    std::lock_guard<std::mutex> g(ctx->stats_mu);
    ctx->mate_last = agg;
    return BSW_OK;
}

int bsw_mate_last_stats(bsw_ctx_t *ctx, bsw_mate_stats_t *out)
{
    if (!ctx || !out) return BSW_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->stats_mu);
    *out = ctx->mate_last;
    return BSW_OK;
}

int bsw_ksw_global2_device(bsw_ctx_t *ctx, SeqPair *d_pairs, const uint8_t *d_ref, const uint8_t *d_qer,
                           int32_t n, uint32_t *d_cigar, int32_t cigar_stride, int32_t *d_n_cigar,
                           void *stream)
{
    if (!ctx || n < 0 || cigar_stride < 0 || (n > 0 && (!d_pairs || !d_ref || !d_qer)) ||
        (n > 0 && cigar_stride > 0 && (!d_cigar || !d_n_cigar)))
        return BSW_E_INVAL;
    if (n == 0) return BSW_OK;
    bsw::GlobParams gp;
    bsw::make_glob_params(ctx->params, ctx->glob_band, gp);
    bsw::DeviceCtx &dc = *ctx->devs[0];
    int rc = BSW_OK;
    auto slot = dc.acquire(rc);
    if (!slot) return rc;
    rc = [&]() -> int {
        BSW_TRY(hipSetDevice(dc.device));
        hipStream_t st = stream ? (hipStream_t)stream : slot->stream;
        bsw_global_stats_t gs;
        const int r = bsw::glob_device(gp, *slot, d_pairs, d_ref, d_qer, n, cigar_stride > 0 ? d_cigar : nullptr,
                                       cigar_stride, d_n_cigar, st, &gs);
        if (r) return r;
        std::lock_guard<std::mutex> g(ctx->stats_mu);
        ctx->glob_last = gs;
        return BSW_OK;
    }();
    dc.give_back(std::move(slot), rc);
    return rc;
}

}  // extern "C"

namespace bsw {
// One device's share of a host-buffer global-alignment call (contiguous job range).
static int glob_host_shard(const GlobParams &gp, DeviceCtx &dc, SeqPair *pairs, const uint8_t *seqBufRef,
                           const uint8_t *seqBufQer, int32_t n, uint32_t *cigar, int32_t cigar_stride,
                           int32_t *n_cigar, bsw_global_stats_t *gs)
{
    *gs = bsw_global_stats_t{};
    if (n == 0) return BSW_OK;
    int rc = BSW_OK;
    auto slot = dc.acquire(rc);
    if (!slot) return rc;
    Slot &s = *slot;
    rc = [&]() -> int {
        BSW_TRY(hipSetDevice(dc.device));
        int64_t r_lo = INT64_MAX, r_hi = 0, q_lo = INT64_MAX, q_hi = 0;
        for (int32_t i = 0; i < n; ++i) {
            const SeqPair &p = pairs[i];
            if (p.len1 > 0) { r_lo = std::min<int64_t>(r_lo, p.idr); r_hi = std::max<int64_t>(r_hi, (int64_t)p.idr + p.len1); }
            if (p.len2 > 0) { q_lo = std::min<int64_t>(q_lo, p.idq); q_hi = std::max<int64_t>(q_hi, (int64_t)p.idq + p.len2); }
        }
        if (r_lo == INT64_MAX) r_lo = r_hi = 0;
        if (q_lo == INT64_MAX) q_lo = q_hi = 0;
        const bool want = cigar_stride > 0;
        BSW_TRY(grow(s.d_pairs, s.cap_pairs, (size_t)n));
        BSW_TRY(grow(s.d_ref, s.cap_ref, (size_t)(r_hi - r_lo) + 1));
        BSW_TRY(grow(s.d_qer, s.cap_qer, (size_t)(q_hi - q_lo) + 1));
        if (want) {
            BSW_TRY(grow(s.d_gcig, s.cap_gcig, (size_t)n * (size_t)cigar_stride));
            BSW_TRY(grow(s.d_gncig, s.cap_gncig, (size_t)n));
        }
        BSW_TRY(hipMemcpyAsync(s.d_pairs, pairs, (size_t)n * sizeof(SeqPair), hipMemcpyHostToDevice, s.stream));
        if (r_hi > r_lo) BSW_TRY(hipMemcpyAsync(s.d_ref, seqBufRef + r_lo, (size_t)(r_hi - r_lo), hipMemcpyHostToDevice, s.stream));
        if (q_hi > q_lo) BSW_TRY(hipMemcpyAsync(s.d_qer, seqBufQer + q_lo, (size_t)(q_hi - q_lo), hipMemcpyHostToDevice, s.stream));
        int r = glob_device(gp, s, s.d_pairs, s.d_ref - r_lo, s.d_qer - q_lo, n, want ? s.d_gcig : nullptr,
                            cigar_stride, want ? s.d_gncig : nullptr, s.stream, gs);
        if (r) return r;
        BSW_TRY(hipMemcpyAsync(pairs, s.d_pairs, (size_t)n * sizeof(SeqPair), hipMemcpyDeviceToHost, s.stream));
        if (want) {
            BSW_TRY(hipMemcpyAsync(cigar, s.d_gcig, (size_t)n * cigar_stride * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
            BSW_TRY(hipMemcpyAsync(n_cigar, s.d_gncig, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, s.stream));
        }
        BSW_TRY(hipStreamSynchronize(s.stream));
        return BSW_OK;
    }();
    dc.give_back(std::move(slot), rc);
    return rc;
}
}  // namespace bsw

extern "C" {

int bsw_ksw_global2(bsw_ctx_t *ctx, SeqPair *pairs, const uint8_t *seqBufRef, const uint8_t *seqBufQer,
                    int32_t n, uint32_t *cigar, int32_t cigar_stride, int32_t *n_cigar)
{
    if (!ctx || n < 0 || cigar_stride < 0 || (n > 0 && (!pairs || !seqBufRef || !seqBufQer)) ||
        (n > 0 && cigar_stride > 0 && (!cigar || !n_cigar)))
        return BSW_E_INVAL;
    if (n == 0) return BSW_OK;
    for (int32_t i = 0; i < n; ++i)
        if (pairs[i].len1 < 0 || pairs[i].len2 < 0 || pairs[i].len1 > BSW_MAX_LEN || pairs[i].len2 > BSW_MAX_LEN ||
            pairs[i].idr < 0 || pairs[i].idq < 0 || pairs[i].h0 < 0)
            return BSW_E_RANGE;
    bsw::GlobParams gp;
    bsw::make_glob_params(ctx->params, ctx->glob_band, gp);
    std::vector<bsw_global_stats_t> st(ctx->devs.size());
    const int rc = bsw::shard_devices(ctx, n, [&](int d, int32_t a, int32_t b) {
        return bsw::glob_host_shard(gp, *ctx->devs[d], pairs + a, seqBufRef, seqBufQer, b - a,
                                    cigar_stride > 0 ? cigar + (size_t)a * cigar_stride : nullptr, cigar_stride,
                                    cigar_stride > 0 ? n_cigar + a : nullptr, &st[d]);
    });
    if (rc) return rc;
    bsw_global_stats_t agg{};
    for (const auto &x : st) {
        agg.kernel_ms = std::max(agg.kernel_ms, x.kernel_ms);
        agg.n_jobs += x.n_jobs; agg.n_lane += x.n_lane; agg.n_wide += x.n_wide; agg.n_launches += x.n_launches;
        agg.cells += x.cells; agg.z_bytes += x.z_bytes; agg.n_tb_retry += x.n_tb_retry;
    }
    std::lock_guard<std::mutex> g(ctx->stats_mu);
    ctx->glob_last = agg;
    return BSW_OK;
}

int bsw_global_last_stats(bsw_ctx_t *ctx, bsw_global_stats_t *out)
{
    if (!ctx || !out) return BSW_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->stats_mu);
    *out = ctx->glob_last;
    return BSW_OK;
}

int bsw_set_reference(bsw_ctx_t *ctx, const uint8_t *ref, int64_t ref_len)
{
    if (!ctx || ref_len < 0 || (ref_len > 0 && !ref)) return BSW_E_INVAL;
    for (auto &dcp : ctx->devs) {
        bsw::DeviceCtx &dc = *dcp;
        std::unique_lock<std::shared_mutex> g(dc.refmu);   // waits for running extension calls
        BSW_TRY(hipSetDevice(dc.device));
        if (dc.d_refres) (void)hipFree(dc.d_refres);
        dc.d_refres = nullptr;
        dc.refres_len = -1;
        BSW_TRY(hipMalloc((void **)&dc.d_refres, (size_t)ref_len + 64));
        if (ref_len > 0) {
            // on a non-blocking stream of its own: a null-stream copy would order against every
            // blocking (CU-masked) slot stream of the process (DeviceCtx::acquire)
            hipStream_t cs = nullptr;
            BSW_TRY(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
            hipError_t e = hipMemcpyAsync(dc.d_refres, ref, (size_t)ref_len, hipMemcpyHostToDevice, cs);
            if (e == hipSuccess) e = hipStreamSynchronize(cs);
            (void)hipStreamDestroy(cs);
            BSW_TRY(e);
        }
        dc.refres_len = ref_len;
    }
    return BSW_OK;
}

int bsw_extend_seeds_device(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *d_reads,
                            const int64_t *d_read_off, const int32_t *d_read_len, const bsw_seed_t *d_seeds,
                            int32_t n, bsw_alnreg_t *d_out, void *stream)
{
    return bsw::extend_seeds_device_win(ctx, opt, d_reads, d_read_off, d_read_len, d_seeds, nullptr, n, d_out, stream);
}

}  // extern "C"

int bsw::extend_seeds_device_win(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *d_reads,
                                 const int64_t *d_read_off, const int32_t *d_read_len, const bsw_seed_t *d_seeds,
                                 const int64_t *d_win, int32_t n, bsw_alnreg_t *d_out, void *stream)
{
    if (!ctx || !opt || n < 0 || (n > 0 && (!d_reads || !d_read_off || !d_read_len || !d_seeds || !d_out)))
        return BSW_E_INVAL;
    bsw::DeviceCtx &dc = *ctx->devs[0];
    std::shared_lock<std::shared_mutex> refg(dc.refmu);   // the resident reference stays put
    if (!dc.d_refres) return BSW_E_INVAL;
    if (const int rc = bsw::ext_opt_check(opt, dc.refres_len)) return rc;
    if (n == 0) return BSW_OK;
    const auto t0 = std::chrono::steady_clock::now();
    int rc = BSW_OK;
    auto slot = dc.acquire(rc);
    if (!slot) return rc;
    bsw::Slot &s = *slot;
    bsw_ext_stats_t es{};
    rc = [&]() -> int {
        BSW_TRY(hipSetDevice(dc.device));
        hipStream_t st = stream ? (hipStream_t)stream : s.stream;
        const bsw_params_t &p = ctx->params;
        bsw::ExtDevParams xp{};
        xp.w = opt->w; xp.pen_clip5 = opt->pen_clip5; xp.pen_clip3 = opt->pen_clip3; xp.a = p.mat[0];
        xp.o_del = p.o_del; xp.e_del = p.e_del; xp.o_ins = p.o_ins; xp.e_ins = p.e_ins;
        xp.ref_len = dc.refres_len;
        xp.l_pac = opt->l_pac;
        // scan: per-read validation and windows, longest read / window, job counts
        BSW_TRY(bsw::grow(s.d_xwin, s.cap_xwin, 2 * (size_t)n));
        BSW_TRY(bsw::launch_ext_scan(xp, d_read_len, d_seeds, d_win, n, s.d_xwin, s.d_meta, st));
        static_assert(bsw::kExtMetaSpread * 16 <= bsw::kMetaWords, "ext meta fits d_meta");
        BSW_TRY(hipMemcpyAsync(s.h_meta, s.d_meta, bsw::kExtMetaSpread * 16 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        BSW_TRY(hipStreamSynchronize(st));
        int32_t m[5] = {0, 0, 0, 0, 0};
        for (int sl = 0; sl < bsw::kExtMetaSpread; ++sl) {
            const int32_t *v = s.h_meta + sl * 16;
            m[0] = std::max(m[0], v[0]); m[1] |= v[1]; m[2] += v[2]; m[3] += v[3]; m[4] = std::max(m[4], v[4]);
        }
        if (m[1]) return BSW_E_RANGE;                   // per read, as the host form (bsw_ext.cpp)
        es.n_pairs[0] = m[2];
        es.n_pairs[2] = m[3];
        xp.qstride = std::max(m[0], 1);                 // longest seeded read
        xp.tstride = std::max(m[4], 1);                 // longest target window (<= BSW_MAX_LEN)
        // SeqPair idr / idq are int32: chunk so i * tstride stays below 2^31
        const int32_t chunk = (int32_t)std::min<int64_t>(std::min<int64_t>(n, (int64_t)INT32_MAX /
                                                                                  std::max(xp.tstride, xp.qstride) - 1),
                                                         bsw::ext_chunk_cap(ctx));
        BSW_TRY(bsw::grow(s.d_xpairs, s.cap_xpairs, (size_t)chunk));
        BSW_TRY(bsw::grow(s.d_xsub, s.cap_xsub, (size_t)chunk));
        BSW_TRY(bsw::grow(s.d_xst, s.cap_xst, (size_t)chunk));
        BSW_TRY(bsw::grow(s.d_xq, s.cap_xq, (size_t)chunk * xp.qstride));
        BSW_TRY(bsw::grow(s.d_xt, s.cap_xt, (size_t)chunk * xp.tstride));
        if (!s.d_mcells) BSW_TRY(hipMalloc((void **)&s.d_mcells, sizeof(unsigned long long)));
        int32_t *d_cnt = (int32_t *)s.d_mcells;
        for (int32_t a = 0; a < n; a += chunk) {
            const int32_t b = std::min(n, a + chunk);
            for (int left = 1; left >= 0; --left) {
                const int r = bsw::ext_side_device(ctx->kp, s, xp, left, *opt, d_reads, d_read_off + a, d_read_len + a,
                                                   d_seeds + a, s.d_xwin + 2 * (size_t)a, b - a, dc.d_refres,
                                                   d_out + a, d_cnt, st, es);
                if (r) return r;
            }
        }
        BSW_TRY(hipStreamSynchronize(st));
        return BSW_OK;
    }();
    dc.give_back(std::move(slot), rc);
    if (rc) return rc;
    es.engine_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    bsw::set_ext_stats(ctx, es);
    return BSW_OK;
}

extern "C" {

int bsw_split_by_cells(const SeqPair *pairs, int32_t n, int32_t w, int32_t parts, int32_t *cut)
{
    if (n < 0 || w < 0 || parts < 1 || !cut || (n > 0 && !pairs)) return BSW_E_INVAL;
    const std::vector<int32_t> c = bsw::split_by_cells(pairs, n, w, parts);
    std::copy(c.begin(), c.end(), cut);
    return BSW_OK;
}

int bsw_set_option(bsw_ctx_t *ctx, int option, int64_t value)
{
    if (!ctx) return BSW_E_INVAL;
    const bool b01 = value == 0 || value == 1;
    switch (option) {
    case BSW_OPT_GQ32_MAX: if (value < 0 || value > INT32_MAX) return BSW_E_INVAL; ctx->kp.gq32_max = (int32_t)value; return BSW_OK;
    case BSW_OPT_KERNEL8: if (value < 0 || value > 2) return BSW_E_INVAL; ctx->kp.kern8 = (int8_t)value; return BSW_OK;
    case BSW_OPT_FORK: if (!b01) return BSW_E_INVAL; ctx->kp.fork = (int8_t)value; return BSW_OK;
    case BSW_OPT_SORTKEY: if (!b01) return BSW_E_INVAL; ctx->kp.keymode = value ? 2 : 0; return BSW_OK;
    case BSW_OPT_GLOB_BAND: if (!b01) return BSW_E_INVAL; ctx->glob_band = (int)value; return BSW_OK;
    case BSW_OPT_EXT_CHUNK: if (value < 0) return BSW_E_INVAL; ctx->ext_chunk = value; return BSW_OK;
    case BSW_OPT_LONG: if (value < 0 || value > 2) return BSW_E_INVAL; ctx->kp.long_route = (int8_t)value; return BSW_OK;
    case BSW_OPT_HOST_CHUNK: if (value < 1 || value > INT32_MAX) return BSW_E_INVAL; ctx->host_chunk = (int32_t)value; return BSW_OK;
    case BSW_OPT_HOST_PACK: if (value != 2 && value != 4) return BSW_E_INVAL; ctx->host_pack = (int)value; return BSW_OK;
    case BSW_OPT_SMALL_BATCH: if (value < 0 || value > INT32_MAX) return BSW_E_INVAL; ctx->kp.small_batch = (int32_t)value; return BSW_OK;
    case BSW_OPT_MID_BATCH: if (value < 0 || value > INT32_MAX) return BSW_E_INVAL; ctx->kp.mid_batch = (int32_t)value; return BSW_OK;
    case BSW_OPT_GROUP_KERNEL: if (!b01) return BSW_E_INVAL; ctx->kp.group_kernel = (int8_t)value; return BSW_OK;
    case BSW_OPT_SPLIT_MIN: if (value < 0) return BSW_E_INVAL; ctx->split_min = value; return BSW_OK;
    case BSW_OPT_COALESCE: if (value < 0 || value > INT32_MAX) return BSW_E_INVAL; ctx->coalesce = (int32_t)value; return BSW_OK;
    case BSW_OPT_COALESCE_LEADERS:
        if (value < 1 || value > 16) return BSW_E_INVAL;
        for (auto &d : ctx->devs) {
            std::lock_guard<std::mutex> g(d->agg_mu);
            d->agg_leaders_max = (int)value;
        }
        return BSW_OK;
    case BSW_OPT_COALESCE_LINGER:
        if (value < 0 || value > 100000) return BSW_E_INVAL;
        for (auto &d : ctx->devs) {
            std::lock_guard<std::mutex> g(d->agg_mu);
            d->agg_linger_us = (int)value;
        }
        return BSW_OK;
    case BSW_OPT_TEST_MISROUTE: if (!b01) return BSW_E_INVAL; ctx->kp.misroute = (int8_t)value; return BSW_OK;
    case BSW_OPT_TEST_FAIL_ALLOC:
        if (value < 0 || value > 1000000) return BSW_E_INVAL;
        bsw::g_fail_alloc.store((int)value);
        return BSW_OK;
    default: return BSW_E_INVAL;
    }
}

int bsw_last_stats(bsw_ctx_t *ctx, bsw_stats_t *out)
{
    if (!ctx || !out) return BSW_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->stats_mu);
    *out = ctx->last;
    return BSW_OK;
}

const char *bsw_strerror(int code)
{
    switch (code) {
    case BSW_OK: return "ok";
    case BSW_E_INVAL: return "invalid argument";
    case BSW_E_NOMEM: return "out of device or pinned host memory";
    case BSW_E_NODEV: return "no such HIP device";
    case BSW_E_HIP: return "HIP runtime error";
    case BSW_E_RANGE: return "pair exceeds supported lengths";
    default: return "unknown error";
    }
}

int bsw_abi_version(void) { return BSW_ABI_VERSION; }

}  // extern "C"
