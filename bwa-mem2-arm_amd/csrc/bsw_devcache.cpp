// bsw_devcache.cpp -- see bsw_devcache.h.
#include "bsw_devcache.h"
#include <map>
#include <mutex>
#include <vector>

namespace bsw {

namespace {

constexpr size_t kDevCacheMax = (size_t)16 << 30;     // idle bytes kept per device
constexpr int kMaxDev = 64;

struct DevCache {
    std::mutex mu;
    std::multimap<size_t, void *> free;               // size class -> blocks
    size_t idle = 0;
    std::vector<StreamLease> streams;
};

DevCache &cache(int device)
{
    static DevCache c[kMaxDev];
    return c[(unsigned)device % kMaxDev];
}

size_t size_class(size_t b)
{
    size_t c = 256;
    while (c < b) c <<= 1;
    return c;
}

}  // namespace

hipError_t devcache_get(int device, size_t bytes, void **out)
{
    const size_t c = size_class(bytes);
    DevCache &d = cache(device);
    {
        std::lock_guard<std::mutex> g(d.mu);
        auto it = d.free.find(c);
        if (it != d.free.end()) {
            *out = it->second;
            d.free.erase(it);
            d.idle -= c;
            return hipSuccess;
        }
    }
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return e;
    e = hipMalloc(out, c);
    if (e == hipErrorOutOfMemory) {                   // drop the idle blocks and retry once
        std::lock_guard<std::mutex> g(d.mu);
        for (auto &kv : d.free) (void)hipFree(kv.second);
        d.free.clear();
        d.idle = 0;
        (void)hipGetLastError();
        e = hipMalloc(out, c);
    }
    return e;
}

void devcache_put(int device, void *p, size_t bytes)
{
    if (!p) return;
    const size_t c = size_class(bytes);
    DevCache &d = cache(device);
    std::lock_guard<std::mutex> g(d.mu);
    if (d.idle + c > kDevCacheMax) {
        (void)hipSetDevice(device);
        (void)hipFree(p);
        return;
    }
    d.free.emplace(c, p);
    d.idle += c;
}

hipError_t stream_lease(int device, StreamLease &out)
{
    DevCache &d = cache(device);
    {
        std::lock_guard<std::mutex> g(d.mu);
        if (!d.streams.empty()) {
            out = d.streams.back();
            d.streams.pop_back();
            return hipSuccess;
        }
    }
    out = StreamLease{};
    out.device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&out.s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipHostMalloc((void **)&out.h, 4 * sizeof(int32_t), 0);
    if (e != hipSuccess) {
        if (out.s) (void)hipStreamDestroy(out.s);
        out = StreamLease{};
    }
    return e;
}

void stream_return(StreamLease &l)
{
    if (!l.s) return;
    DevCache &d = cache(l.device);
    std::lock_guard<std::mutex> g(d.mu);
    d.streams.push_back(l);
    l = StreamLease{};
}

}  // namespace bsw
