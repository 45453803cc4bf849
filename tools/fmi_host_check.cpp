// Host-side run of the SMEM kernel's per-read code (smem_read, compiled __host__ __device__) over
// a host-only index: a CPU debugging harness for bsw_fmi.hip's state machine (never shipped).
//   fmi_host_check ref.bin reads.bin off.bin len.bin cap out_mems.bin out_cnt.bin
#include <hip/hip_runtime.h>
#undef __device__
#define __device__ __attribute__((host)) __attribute__((device))
#include "../bwa-mem2-arm_amd/csrc/bsw_fmi.hip"
#include <cstdio>
static std::vector<char> slurp(const char *p)
{
    FILE *f = fopen(p, "rb");
    std::vector<char> b;
    if (!f) return b;
    fseek(f, 0, SEEK_END);
    b.resize(ftell(f));
    fseek(f, 0, SEEK_SET);
    if (fread(b.data(), 1, b.size(), f) != b.size()) b.clear();
    fclose(f);
    return b;
}
int main(int argc, char **argv)
{
    if (argc < 8) return 2;
    auto ref = slurp(argv[1]), reads = slurp(argv[2]), off = slurp(argv[3]), len = slurp(argv[4]);
    const int cap = atoi(argv[5]);
    bsw_fmi_t *f = nullptr;
    if (bsw_fmi_build((const uint8_t *)ref.data(), (int64_t)ref.size(), -1, &f) != 0) return 3;
    const int n = (int)(len.size() / 4);
    const int32_t *L = (const int32_t *)len.data();
    int maxlen = 0;
    for (int i = 0; i < n; ++i) maxlen = std::max(maxlen, L[i]);
    const int scap = maxlen + 1;
    std::vector<uint4> scratch((size_t)2 * scap * n);
    std::vector<bsw_bwtintv_t> mems((size_t)n * cap);
    std::vector<int32_t> cnt(n);
    MemOpt mo{19, 10, 20, (int)(19 * 1.5f + .499)};
    int err = 0;
    for (int t = 0; t < n; ++t)
        err |= smem_read(f->dv, mo, (const uint8_t *)reads.data(), (const int64_t *)off.data(), L, 0, n, t,
                         scratch.data(), scap, mems.data(), cap, cnt.data());
    FILE *o = fopen(argv[6], "wb");
    fwrite(mems.data(), sizeof(bsw_bwtintv_t), mems.size(), o);
    fclose(o);
    o = fopen(argv[7], "wb");
    fwrite(cnt.data(), 4, n, o);
    fclose(o);
    printf("err %d\n", err);
    bsw_fmi_destroy(f);
    return 0;
}
