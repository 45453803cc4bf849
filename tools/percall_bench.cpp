// percall_bench.cpp -- the drop-in regime measured the way upstream calls it: C++ kt_for-style
// worker threads issuing getScores16-sized host-buffer calls through the C ABI (bsw_get_scores),
// no Python in the loop.  C2-shaped pairs from libbsw_synth.so (splitmix64, seed 42).
//   percall_bench [pairs_total] [threads] [sizes...]
// For every call size: median single-caller latency (1 thread, 200 calls after warm-up) and the
// aggregate rate of `threads` concurrent callers (each issuing calls back to back over its own
// slice of the batch for 0.5 s after an untimed warm-up of every caller), with cross-call
// coalescing (default) and without (BSW_OPT_COALESCE = 0) interleaved on / off / on / off, min
// and max of each kept; one JSON line on stdout.  Outputs are checked against a whole-batch call
// (bit-identical required).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <thread>
#include <ucontext.h>
#include <unistd.h>
#include <vector>
#include "../include/bsw.h"

// Fault diagnostics (PERCALL_SEGV_LOG=<file>): on SIGSEGV / SIGBUS write the faulting address,
// the faulting PC, every backtrace frame with the object that holds it (dladdr: file, load base,
// offset, nearest symbol) and the whole /proc/self/maps to <file>, then die with the signal.
// Replaces whatever handler a profiler installed before main (rocprofv3's glog handler prints
// bare addresses); not async-signal-safe, which does not matter on the way down.
static const char *g_segv_log = nullptr;
static void put_addr(FILE *f, const char *what, void *a)
{
    Dl_info di{};
    if (a && dladdr(a, &di) && di.dli_fname)
        fprintf(f, "%s %p  %s + 0x%lx  (%s + 0x%lx)\n", what, a, di.dli_fname,
                (unsigned long)((char *)a - (char *)di.dli_fbase), di.dli_sname ? di.dli_sname : "?",
                di.dli_saddr ? (unsigned long)((char *)a - (char *)di.dli_saddr) : 0ul);
    else
        fprintf(f, "%s %p  (no object: not inside any loaded image)\n", what, a);
}
static void on_fault(int sig, siginfo_t *si, void *uc_)
{
    FILE *f = fopen(g_segv_log, "w");
    if (!f) f = stderr;
    const ucontext_t *uc = (const ucontext_t *)uc_;
    fprintf(f, "signal %d code %d tid %ld\n", sig, si->si_code, (long)gettid());
    put_addr(f, "fault address", si->si_addr);
    put_addr(f, "faulting pc  ", (void *)uc->uc_mcontext.gregs[REG_RIP]);
    void *fr[64];
    const int n = backtrace(fr, 64);
    for (int k = 0; k < n; ++k) {
        char w[32];
        snprintf(w, sizeof w, "frame %2d     ", k);
        put_addr(f, w, fr[k]);
    }
    fprintf(f, "---- /proc/self/maps\n");
    if (FILE *m = fopen("/proc/self/maps", "r")) {
        char line[512];
        while (fgets(line, sizeof line, m)) fputs(line, f);
        fclose(m);
    }
    if (f != stderr) fclose(f);
    fprintf(stderr, "percall_bench: signal %d at %p, diagnostics in %s\n", sig, si->si_addr, g_segv_log);
    signal(sig, SIG_DFL);
    raise(sig);
}

extern "C" {
typedef struct { uint64_t seed; int32_t tlen, qlen, h0_lo, h0_hi; double p_sub, p_indel, p_unrelated, p_n; } synth_cfg;
void bsw_synth_default(synth_cfg *c);
void bsw_synth_batch(const synth_cfg *c, int64_t base, int32_t n, SeqPair *pairs, uint8_t *ref, uint8_t *qer);
}

using Clock = std::chrono::steady_clock;
static double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

int main(int argc, char **argv)
{
    if ((g_segv_log = getenv("PERCALL_SEGV_LOG"))) {
        struct sigaction sa{};
        sa.sa_sigaction = on_fault;
        sa.sa_flags = SA_SIGINFO;
        sigaction(SIGSEGV, &sa, nullptr);
        sigaction(SIGBUS, &sa, nullptr);
    }
    const int32_t N = argc > 1 ? atoi(argv[1]) : 1000000;
    const int T = argc > 2 ? atoi(argv[2]) : 8;
    std::vector<int32_t> sizes;
    for (int k = 3; k < argc; ++k) sizes.push_back(atoi(argv[k]));
    if (sizes.empty()) sizes = {1000, 10000, 100000};
    synth_cfg c;
    bsw_synth_default(&c);
    std::vector<SeqPair> pairs(N);
    std::vector<uint8_t> ref((size_t)N * c.tlen), qer((size_t)N * c.qlen);
    bsw_synth_batch(&c, 0, N, pairs.data(), ref.data(), qer.data());
    bsw_params_t p;
    bsw_params_default(&p);
    bsw_ctx_t *ctx = nullptr;
    if (bsw_create(&p, 0, 1, &ctx) != BSW_OK) { fprintf(stderr, "bsw_create failed\n"); return 2; }
    if (const char *l = getenv("PERCALL_LEADERS")) bsw_set_option(ctx, BSW_OPT_COALESCE_LEADERS, atoi(l));
    if (const char *g = getenv("PERCALL_GROUP")) bsw_set_option(ctx, BSW_OPT_GROUP_KERNEL, atoi(g));
    if (const char *b = getenv("PERCALL_SMALL")) bsw_set_option(ctx, BSW_OPT_SMALL_BATCH, atoi(b));
    if (const char *b = getenv("PERCALL_GQ32_MAX")) bsw_set_option(ctx, BSW_OPT_GQ32_MAX, atoi(b));
    if (const char *b = getenv("PERCALL_LINGER")) bsw_set_option(ctx, BSW_OPT_COALESCE_LINGER, atoi(b));
    std::vector<SeqPair> want = pairs;
    if (bsw_get_scores(ctx, want.data(), ref.data(), qer.data(), N, 100, 16) != BSW_OK) return 3;
    printf("{\"tool\": \"percall_bench\", \"threads\": %d, \"pairs\": %d, \"seconds_per_run\": 0.5, "
           "\"order\": \"per size: 1-caller latency, then %d-caller runs interleaved coalescing on/off/on/off, each "
           "after an untimed warm-up of every caller\", \"curve\": [", T, N, T);
    bool first = true;
    std::atomic<long> bad{0};
    const int32_t co_on = getenv("PERCALL_COALESCE") ? atoi(getenv("PERCALL_COALESCE")) : 8192;   // the library default
    // T concurrent callers, each over its own contiguous slice, calls back to back for `secs_run`;
    // returns M pairs / s
    auto callers = [&](int32_t m, double secs_run) {
        std::atomic<long> done{0};
        std::vector<std::thread> th;
        const int32_t slice = N / T;
        const auto t0 = Clock::now();
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                std::vector<SeqPair> b(m);
                for (int32_t k = 0;; ++k) {
                    const int32_t a = t * slice + (int32_t)(((int64_t)k * m) % (slice - m + 1));
                    std::copy(pairs.begin() + a, pairs.begin() + a + m, b.begin());
                    if (bsw_get_scores(ctx, b.data(), ref.data(), qer.data(), m, 100, 16) != BSW_OK) { bad += 1000000; return; }
                    for (int32_t i = 0; i < m; ++i) bad += memcmp(&b[i].score, &want[a + i].score, 24) != 0;
                    done.fetch_add(m);
                    if (secs(t0, Clock::now()) > secs_run) break;
                }
            });
        for (auto &x : th) x.join();
        return done.load() / secs(t0, Clock::now()) / 1e6;
    };
    for (int32_t m : sizes) {
        if (m > N / T) continue;
        // one caller: median latency (coalescing on: a lone caller leads its own batch at once)
        bsw_set_option(ctx, BSW_OPT_COALESCE, co_on);
        std::vector<SeqPair> buf(pairs.begin(), pairs.begin() + m);
        std::vector<double> lat;
        for (int k = 0; k < 203; ++k) {
            const int32_t a = (int32_t)(((int64_t)k * m) % (N - m + 1));
            std::copy(pairs.begin() + a, pairs.begin() + a + m, buf.begin());
            const auto t0 = Clock::now();
            if (bsw_get_scores(ctx, buf.data(), ref.data(), qer.data(), m, 100, 16) != BSW_OK) return 4;
            if (k >= 3) lat.push_back(secs(t0, Clock::now()));
            for (int32_t i = 0; i < m; ++i) bad += memcmp(&buf[i].score, &want[a + i].score, 24) != 0;
        }
        std::sort(lat.begin(), lat.end());
        const double med = lat[lat.size() / 2];
        // T callers, coalescing on / off interleaved A-B-A-B, each run after a warm-up of every
        // caller (its slots, the coalescing leaders' buffers at this size)
        std::vector<double> r[2];
        for (int rep = 0; rep < 2; ++rep)
            for (int co = 1; co >= 0; --co) {
                bsw_set_option(ctx, BSW_OPT_COALESCE, co ? co_on : 0);
                callers(m, 0.05);
                r[co].push_back(callers(m, 0.5));
            }
        auto stat = [](std::vector<double> v) {
            std::sort(v.begin(), v.end());
            char o[256];
            snprintf(o, sizeof o, "{\"median\": %.3f, \"min\": %.3f, \"max\": %.3f, \"runs\": [%.3f, %.3f]}",
                     (v.front() + v.back()) / 2, v.front(), v.back(), v[0], v[1]);
            return std::string(o);
        };
        printf("%s{\"pairs_per_call\": %d, \"latency_ms_median\": %.3f, \"M_pairs_per_s_1_caller\": %.3f, "
               "\"M_pairs_per_s_%d_callers_coalescing\": %s, \"M_pairs_per_s_%d_callers_no_coalescing\": %s}",
               first ? "" : ", ", m, med * 1e3, m / med / 1e6, T, stat(r[1]).c_str(), T, stat(r[0]).c_str());
        first = false;
        fflush(stdout);
    }
    bsw_set_option(ctx, BSW_OPT_COALESCE, co_on);
    // PERCALL_MAPS_LOG=<file>: this process's mappings at the end of a clean run (to place the
    // addresses of an earlier run's fault: the libraries' load order and sizes are the same, so
    // their offsets from libbsw_hip.so's load base carry over; ASLR moves only the whole block)
    if (const char *ml = getenv("PERCALL_MAPS_LOG"))
        if (FILE *f = fopen(ml, "w")) {
            put_addr(f, "bsw_get_scores", (void *)&bsw_get_scores);
            if (FILE *m = fopen("/proc/self/maps", "r")) {
                char line[512];
                while (fgets(line, sizeof line, m)) fputs(line, f);
                fclose(m);
            }
            fclose(f);
        }
    printf("],\"outputs_identical\": %s}\n", bad.load() == 0 ? "true" : "false");
    bsw_destroy(ctx);
    return bad.load() == 0 ? 0 : 5;
}
