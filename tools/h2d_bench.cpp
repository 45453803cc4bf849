// PCIe copy-rate probe on the GPU box: pinned (hipHostMalloc) H2D / D2H of 512 MB as one copy,
// and split over 2 / 4 streams; pageable H2D for comparison.  Output: one JSON line per case.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
// zero-copy "pull": a kernel streams pinned host memory over PCIe into HBM (16-B loads, many in flight)
__global__ void pull_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
int main()
{
    const size_t B = (size_t)512 << 20;
    void *h = nullptr, *d = nullptr;
    CK(hipHostMalloc(&h, B, 0));
    CK(hipMalloc(&d, B));
    memset(h, 1, B);
    void *pg = malloc(B);
    memset(pg, 2, B);
    hipStream_t st[4];
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto run = [&](const char *name, int ns, bool h2d, void *src) {
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipDeviceSynchronize());
            auto t0 = std::chrono::steady_clock::now();
            for (int k = 0; k < ns; ++k) {
                const size_t a = B * k / ns, b = B * (k + 1) / ns;
                if (h2d) CK(hipMemcpyAsync((char *)d + a, (char *)src + a, b - a, hipMemcpyHostToDevice, st[k]));
                else CK(hipMemcpyAsync((char *)src + a, (char *)d + a, b - a, hipMemcpyDeviceToHost, st[k]));
            }
            for (int k = 0; k < ns; ++k) CK(hipStreamSynchronize(st[k]));
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (rep == 3) printf("{\"case\": \"%s\", \"streams\": %d, \"GBps\": %.2f}\n", name, ns, B / s / 1e9);
        }
    };
    run("pinned_h2d", 1, true, h); run("pinned_h2d", 2, true, h); run("pinned_h2d", 4, true, h);
    run("pinned_d2h", 1, false, h); run("pinned_d2h", 2, false, h);
    run("pageable_h2d", 1, true, pg);
    {
        void *hd = nullptr;
        CK(hipHostGetDevicePointer(&hd, h, 0));
        for (int grid : {512, 1024, 2048, 4096}) {
            double best = 0;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                hipLaunchKernelGGL(pull_kernel, dim3(grid), dim3(256), 0, st[0], (const uint4 *)hd, (uint4 *)d, B / 16);
                CK(hipStreamSynchronize(st[0]));
                const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                best = std::max(best, B / s / 1e9);
            }
            printf("{\"case\": \"pull_kernel_h2d\", \"grid\": %d, \"GBps\": %.2f}\n", grid, best);
        }
        if (((unsigned char *)d)[0] == 0) {}   // keep d
        std::vector<unsigned char> chk(64);
        CK(hipMemcpy(chk.data(), d, 64, hipMemcpyDeviceToHost));
        printf("{\"case\": \"pull_check\", \"ok\": %d}\n", chk[0] == 1 && chk[63] == 1);
    }
    // host memcpy into pinned memory (the staging step), 1 thread
    auto t0 = std::chrono::steady_clock::now();
    memcpy(h, pg, B);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"case\": \"memcpy_to_pinned_1thread\", \"GBps\": %.2f}\n", B / s / 1e9);
    return 0;
}
