// bsw_devcache.h -- per-device caches of the scratch that the chain / seeding entry points
// used to hipMalloc and hipFree on every call (C1: ~20 allocations per mem_chain2aln call, each
// a driver round trip of tens of microseconds -- most of a 10K-read call's time).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace bsw {

// A device block of at least `bytes` (size classes: powers of two from 256 B); hipMalloc on a
// miss.  Blocks go back with devcache_put(device, p, bytes) once no queued work uses them; the
// cache frees beyond kDevCacheMax idle bytes per device.
hipError_t devcache_get(int device, size_t bytes, void **out);
void devcache_put(int device, void *p, size_t bytes);

// A non-blocking stream plus a small pinned host word array (readbacks), reused across calls.
struct StreamLease {
    int device = -1;
    hipStream_t s = nullptr;
    int32_t *h = nullptr;            // 4 pinned int32 words
};
hipError_t stream_lease(int device, StreamLease &out);
void stream_return(StreamLease &l);  // the caller has synchronised l.s

// One call's device scratch: get() takes cached blocks, the destructor synchronises `stream`
// (if set: nothing queued may still use the blocks) and returns them.
struct CachedBufs {
    static constexpr int kMax = 24;
    int device;
    hipStream_t stream = nullptr;
    void *p[kMax] = {};
    size_t sz[kMax] = {};
    int n = 0;
    explicit CachedBufs(int d) : device(d) {}
    template <class T>
    hipError_t get(T *&out, size_t count)
    {
        if (n == kMax) return hipErrorInvalidValue;
        void *q = nullptr;
        const size_t b = (count > 0 ? count : 1) * sizeof(T);
        const hipError_t e = devcache_get(device, b, &q);
        if (e == hipSuccess) { p[n] = q; sz[n] = b; ++n; out = (T *)q; }
        return e;
    }
    ~CachedBufs()
    {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        for (int k = 0; k < n; ++k) devcache_put(device, p[k], sz[k]);
    }
};

}  // namespace bsw
