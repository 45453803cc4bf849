// bandedSWA_gpu.h -- header-only drop-in for upstream bwa-mem2's `BandedPairWiseSW`
// (src/bandedSWA.h), backed by the MI355X engine through the C ABI in bsw.h.
//
// Same class name, constructor and member signatures the upstream callers use:
//   ctor      BandedPairWiseSW(o_del, e_del, o_ins, e_ins, zdrop, end_bonus, mat, w_match,
//             w_mismatch, numThreads)        -- call site docs-archive/INTEGRATION_COMPLETE.md:61-63
//   getScores16 / getScores8 (SeqPair*, uint8_t* seqBufRef, uint8_t* seqBufQer,
//             int32_t numPairs, uint16_t numThreads, int32_t w)
//                                            -- docs-archive/WEEK1_WRAPPER_COMPLETE.md:259-269
//   scalarBandedSWAWrapper / scalarBandedSWA -- upstream's scalar path [UPSTREAM-RECALL]
// so bwamem.cpp (mem_chain2aln_across_reads_V2) compiles unchanged after swapping the
// include.  Every entry point runs on the GPU: there is no CPU fallback.  Upstream's error
// convention is kept: void members, and on any engine error a message on stderr followed
// by exit(EXIT_FAILURE) (style of docs-archive/ARM-BATCHED-SAM-PLAN.md:93-110).
// numThreads is accepted for signature compatibility; concurrency comes from the device.
// Environment: BSW_GPUS = number of GPUs (default 1), BSW_DEVICE0 = first HIP device index
//              (default 0): devices [BSW_DEVICE0, BSW_DEVICE0 + BSW_GPUS); or BSW_GPU_MAP =
//              "d0,d1,..." = the HIP device of each logical device (repeats allowed: the
//              rehearsal of an n-GPU node on a smaller box).  With several devices a
//              getScores* call of fewer than 131072 pairs runs whole on the least-busy device
//              and larger ones are split by band cells (bsw.h, BSW_OPT_SPLIT_MIN).
#ifndef BANDEDSWA_GPU_H
#define BANDEDSWA_GPU_H

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "bsw.h"
#include "bsw_batch.h"

#ifndef MAX_SEQ_LEN8
#define MAX_SEQ_LEN8 BSW_MAX_SEQ_LEN8
#endif
#ifndef AMBIG
#define AMBIG BSW_AMBIG
#endif

class BandedPairWiseSW {
public:
    BandedPairWiseSW(const int o_del, const int e_del, const int o_ins, const int e_ins,
                     const int zdrop, const int end_bonus, const int8_t *mat_,
                     const int8_t w_match, const int8_t w_mismatch, int numThreads)
    {
        (void)numThreads;
        bsw_params_t p;
        bsw_params_default(&p);
        p.o_del = o_del; p.e_del = e_del; p.o_ins = o_ins; p.e_ins = e_ins;
        p.zdrop = zdrop; p.end_bonus = end_bonus;
        if (mat_) memcpy(p.mat, mat_, 25);
        p.w_match = w_match; p.w_mismatch = w_mismatch; p.w_ambig = -1;
        const char *g = getenv("BSW_GPUS"), *d0 = getenv("BSW_DEVICE0"), *map = getenv("BSW_GPU_MAP");
        const int ngpu = g ? atoi(g) : 1, dev0 = d0 ? atoi(d0) : 0;
        if (map && *map) {
            int devs[256], nd = 0;
            for (const char *c = map; *c && nd < 256;) {
                devs[nd++] = atoi(c);
                while (*c && *c != ',') ++c;
                if (*c == ',') ++c;
            }
            check(bsw_create_on(&p, devs, nd, &ctx_), "bsw_create_on (BSW_GPU_MAP)");
        } else {
            check(bsw_create(&p, dev0, ngpu > 0 ? ngpu : 1, &ctx_), "bsw_create");
        }
        params_ = p;
        record_ = getenv("BSW_RECORD");   // capture every batch as <prefix>.<n>.bswb (bsw_batch.h)
    }
    ~BandedPairWiseSW() { bsw_destroy(ctx_); }
    BandedPairWiseSW(const BandedPairWiseSW &) = delete;
    BandedPairWiseSW &operator=(const BandedPairWiseSW &) = delete;

    void getScores16(SeqPair *pairArray, uint8_t *seqBufRef, uint8_t *seqBufQer, int32_t numPairs,
                     uint16_t numThreads, int32_t w)
    {
        (void)numThreads;
        check(bsw_get_scores(ctx_, pairArray, seqBufRef, seqBufQer, numPairs, w, 16), "getScores16");
        if (record_) record(pairArray, seqBufRef, seqBufQer, numPairs, w, 16);
    }
    void getScores8(SeqPair *pairArray, uint8_t *seqBufRef, uint8_t *seqBufQer, int32_t numPairs,
                    uint16_t numThreads, int32_t w)
    {
        (void)numThreads;
        check(bsw_get_scores(ctx_, pairArray, seqBufRef, seqBufQer, numPairs, w, 8), "getScores8");
        if (record_) record(pairArray, seqBufRef, seqBufQer, numPairs, w, 8);
    }
    void scalarBandedSWAWrapper(SeqPair *seqPairArray, uint8_t *seqBufRef, uint8_t *seqBufQer,
                                int numPairs, int nthreads, int32_t w)
    {
        (void)nthreads;
        check(bsw_get_scores(ctx_, seqPairArray, seqBufRef, seqBufQer, numPairs, w, 16),
              "scalarBandedSWAWrapper");
    }
    int scalarBandedSWA(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int32_t w,
                        int h0, int *_qle, int *_tle, int *_gtle, int *_gscore, int *_max_off)
    {
        SeqPair sp;
        memset(&sp, 0, sizeof(sp));
        sp.len1 = tlen; sp.len2 = qlen; sp.h0 = h0;
        check(bsw_get_scores(ctx_, &sp, target, query, 1, w, 16), "scalarBandedSWA");
        if (_qle) *_qle = sp.qle;
        if (_tle) *_tle = sp.tle;
        if (_gtle) *_gtle = sp.gtle;
        if (_gscore) *_gscore = sp.gscore;
        if (_max_off) *_max_off = sp.max_off;
        return sp.score;
    }

private:
    // Record a finished batch (outputs included): the byte buffers up to the furthest byte
    // any pair references.  Concurrent kt_for callers get distinct sequence numbers.
    void record(const SeqPair *pairs, const uint8_t *ref, const uint8_t *qer, int32_t n, int32_t w,
                int cell_bits)
    {
        int64_t rb = 0, qb = 0;
        for (int32_t i = 0; i < n; ++i) {
            if ((int64_t)pairs[i].idr + pairs[i].len1 > rb) rb = (int64_t)pairs[i].idr + pairs[i].len1;
            if ((int64_t)pairs[i].idq + pairs[i].len2 > qb) qb = (int64_t)pairs[i].idq + pairs[i].len2;
        }
        const unsigned k = __atomic_fetch_add(&seq_, 1u, __ATOMIC_RELAXED);
        char path[4096];
        snprintf(path, sizeof(path), "%s.%06u.bswb", record_, k);
        check(bswb_write(path, &params_, w, cell_bits, 1, pairs, n, ref, rb, qer, qb), "BSW_RECORD");
    }
    // reached only after the engine's own recovery (bsw.h, bsw_get_scores: a failed device run is
    // rerun on fresh buffers, on the context's other devices, then in halves) has also failed
    static void check(int rc, const char *what)
    {
        if (rc != BSW_OK) {
            fprintf(stderr, "[BandedPairWiseSW] %s failed: %s (%d)\n", what, bsw_strerror(rc), rc);
            exit(EXIT_FAILURE);
        }
    }
    bsw_ctx_t *ctx_ = nullptr;
    bsw_params_t params_{};
    const char *record_ = nullptr;
    unsigned seq_ = 0;
};

#endif  // BANDEDSWA_GPU_H
