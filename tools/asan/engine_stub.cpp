// engine_stub.cpp -- host-only stand-in for the GPU engine hooks bsw_ext.cpp calls
// (csrc/bsw_internal.h), so the extension job builder / interpreter / chain rounds can run
// under AddressSanitizer + UBSan without a GPU (`make asan`).  scores_eb scores each SeqPair
// with the CPU oracle's ksw_extend2 (oracle/ksw_ext_ref.c); everything else is bookkeeping.
// TEST INFRASTRUCTURE: never part of the product library.
#include <cstring>
#include <mutex>
#include "../../bwa-mem2-arm_amd/csrc/bsw_internal.h"

extern "C" int oracle_ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
                                  const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                                  int end_bonus, int zdrop, int h0, int *qle, int *tle, int *gtle, int *gscore,
                                  int *max_off);

struct bsw_ctx {
    bsw_params_t params;
    bsw_ext_stats_t ext{};
    bsw_chain_stats_t chain{};
    std::mutex mu;
};

extern "C" bsw_ctx_t *stub_ctx_create(const bsw_params_t *p)
{
    auto *c = new bsw_ctx();
    c->params = *p;
    return c;
}
extern "C" void stub_ctx_destroy(bsw_ctx_t *c) { delete c; }

namespace bsw {
int scores_eb(bsw_ctx_t *ctx, int32_t end_bonus, SeqPair *pairs, const uint8_t *ref, const uint8_t *qer, int32_t n,
              int32_t w, int cell_bits, bsw_stats_t *st)
{
    (void)cell_bits;
    const bsw_params_t &p = ctx->params;
    for (int32_t i = 0; i < n; ++i) {
        SeqPair &s = pairs[i];
        if (s.len1 < 0 || s.len2 < 0 || s.len1 > BSW_MAX_LEN || s.len2 > BSW_MAX_LEN) return BSW_E_RANGE;
        int qle, tle, gtle, gscore, max_off;
        s.score = oracle_ksw_extend2(s.len2, qer + s.idq, s.len1, ref + s.idr, 5, p.mat, p.o_del, p.e_del, p.o_ins,
                                     p.e_ins, w, end_bonus, p.zdrop, s.h0, &qle, &tle, &gtle, &gscore, &max_off);
        s.qle = qle; s.tle = tle; s.gtle = gtle; s.gscore = gscore; s.max_off = max_off;
    }
    if (st) *st = bsw_stats_t{};
    return BSW_OK;
}
void ctx_params(const bsw_ctx_t *ctx, bsw_params_t *out) { *out = ctx->params; }
int ctx_device(const bsw_ctx_t *) { return 0; }
int64_t ctx_refres_len(bsw_ctx_t *) { return -1; }
void *pinned_acquire(bsw_ctx_t *, int, size_t) { return nullptr; }     // builder falls back to heap
void pinned_release(bsw_ctx_t *, int) {}
void set_ext_stats(bsw_ctx_t *ctx, const bsw_ext_stats_t &s) { std::lock_guard<std::mutex> g(ctx->mu); ctx->ext = s; }
int get_ext_stats(bsw_ctx_t *ctx, bsw_ext_stats_t *out) { std::lock_guard<std::mutex> g(ctx->mu); *out = ctx->ext; return 0; }
int64_t ext_chunk_cap(const bsw_ctx_t *) { return 7777; }               // exercise the chunked path
void set_chain_stats(bsw_ctx_t *ctx, const bsw_chain_stats_t &s) { std::lock_guard<std::mutex> g(ctx->mu); ctx->chain = s; }
int get_chain_stats(bsw_ctx_t *ctx, bsw_chain_stats_t *out) { std::lock_guard<std::mutex> g(ctx->mu); *out = ctx->chain; return 0; }
}  // namespace bsw
