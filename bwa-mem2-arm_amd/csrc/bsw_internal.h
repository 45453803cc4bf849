// bsw_internal.h -- engine hooks shared by the C ABI translation units (not installed).
#pragma once
#include "../../include/bsw.h"
#include "../../include/bsw_ext.h"
#include <cstdint>
#include <vector>

namespace bsw {
// bsw_get_scores with a per-call end_bonus (LEFT uses pen_clip5, RIGHT pen_clip3) and the
// call's stats returned instead of stored.
int scores_eb(bsw_ctx_t *ctx, int32_t end_bonus, SeqPair *pairs, const uint8_t *ref,
              const uint8_t *qer, int32_t n, int32_t w, int cell_bits, bsw_stats_t *st);
void ctx_params(const bsw_ctx_t *ctx, bsw_params_t *out);
int ctx_device(const bsw_ctx_t *ctx);          // HIP device of the context's first device slot pool
int64_t ctx_refres_len(bsw_ctx_t *ctx);        // length of the resident reference (-1: none)
// Per-context pinned host staging buffer `which` (0, 1) of at least `bytes`: DMA-speed H2D for
// the extension pipeline's code buffers.  Returns nullptr when another call holds it (the
// caller then uses pageable memory); release with pinned_release.
void *pinned_acquire(bsw_ctx_t *ctx, int which, size_t bytes);
void pinned_release(bsw_ctx_t *ctx, int which);
void set_ext_stats(bsw_ctx_t *ctx, const bsw_ext_stats_t &s);
int64_t ext_chunk_cap(const bsw_ctx_t *ctx);   // reads per extension chunk (BSW_OPT_EXT_CHUNK)
int get_ext_stats(bsw_ctx_t *ctx, bsw_ext_stats_t *out);
void set_chain_stats(bsw_ctx_t *ctx, const bsw_chain_stats_t &s);
int get_chain_stats(bsw_ctx_t *ctx, bsw_chain_stats_t *out);
// bsw_ext_opt_t / seed checks shared by the host and device extension forms (bsw_ext.cpp)
int ext_opt_check(const bsw_ext_opt_t *opt, int64_t ref_len);
bool ext_seed_ok(const bsw_ext_opt_t *opt, const bsw_seed_t &s, int32_t l, int64_t ref_len);
// bsw_extend_seeds_device with each job's target window given (d_win[2j], d_win[2j + 1]: the
// chain's window, mem_chain2aln) or computed per seed (d_win == nullptr)
int extend_seeds_device_win(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *d_reads,
                            const int64_t *d_read_off, const int32_t *d_read_len, const bsw_seed_t *d_seeds,
                            const int64_t *d_win, int32_t n, bsw_alnreg_t *d_out, void *stream);
// mem_chain2aln rounds with every per-read decision on the GPU (bsw_chain.hip): inputs and
// outputs device-resident on the context's first device
int chain_rounds_device(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *d_reads, const int64_t *d_read_off,
                        const int32_t *d_read_len, int32_t n_reads, const bsw_seed_t *d_seeds,
                        const int32_t *d_sr, const int32_t *d_sc, int32_t ns, bsw_alnreg_t *d_out, int32_t *d_ext,
                        bsw_chain_stats_t *cs);
// staging packers (bsw_pack.cpp): nibbles (dst[k] = src[2k] & 15 | (src[2k+1] & 15) << 4) and
// 2-bit codes + exception words (pos0 + k) << 4 | (src[k] & 15) for bytes outside 0..3
void pack_nibbles(uint8_t *dst, const uint8_t *src, size_t nbytes);
void pack_2bit(uint8_t *dst, const uint8_t *src, size_t nbytes, uint32_t pos0, std::vector<uint32_t> &exc);
// host pipeline fast path (bsw_host.cpp host_shard_fast): plan_kernel's schedule key of the
// packed-column class for pairs [0, n) -- (255 - qlen) << 20 | (1 - related) << 19 |
// (63 - tlen / 32) << 13 | (31 - seed identities) << 8 | (255 - h0), identities as the device's
// seed_matches (best of 13 shifts of query[10, 40) against target[4 + s, 34 + s))
void fast_keys(const SeqPair *pairs, int32_t n, const uint8_t *ref, const uint8_t *qer, uint32_t *keys);
// kv[i] = (the bits of keys[i] selected by `vary`, compacted: pext) << 32 | i, for i in [a0, a1)
void compact_keys(const uint32_t *keys, int32_t a0, int32_t a1, uint32_t vary, uint64_t *kv);
}  // namespace bsw
