// bsw_ext_k.h -- launch interface of the device-side extension pipeline (bsw_ext_dev.hip).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "../../include/bsw_seqpair.h"
#include "../../include/bsw_ext.h"

namespace bsw {

struct ExtDevParams {
    int32_t w, pen_clip5, pen_clip3, a;
    int32_t o_del, e_del, o_ins, e_ins;
    int32_t qstride, tstride;           // per-read code-buffer strides
    int64_t ref_len;
    int64_t l_pac;                      // bsw_ext_opt_t::l_pac (0: one-strand reference)
};

struct ExtState {                       // per read, between the phases
    int64_t rmax0, rmax1;               // target window
    int32_t score, prev;                // a->score (h0 of RIGHT), score before the band loop
    int32_t lw, rw;                     // band used per side
};

constexpr int kExtMetaSpread = 32;     // ext_scan writes meta[slot * 16 + k], slot < 32

// validation + target windows (win: given per job, or nullptr: each seed's own) into wout[2n]
hipError_t launch_ext_scan(const ExtDevParams &p, const int32_t *read_len, const bsw_seed_t *seeds, const int64_t *win,
                           int32_t n, int64_t *wout, int32_t *meta, hipStream_t s);
hipError_t launch_ext_build(int left, const ExtDevParams &p, const uint8_t *reads, const int64_t *read_off,
                            const int32_t *read_len, const bsw_seed_t *seeds, const int64_t *win, int32_t n,
                            const uint8_t *ref, ExtState *st, SeqPair *pairs, uint8_t *qbuf, uint8_t *tbuf,
                            bsw_alnreg_t *out, hipStream_t s);
hipError_t launch_ext_retry_mark(const SeqPair *src, SeqPair *sub, ExtState *st, int32_t n, int32_t wt,
                                 int32_t *cnt, hipStream_t s);
hipError_t launch_ext_retry_merge(SeqPair *pairs, const SeqPair *sub, ExtState *st, int32_t n, int32_t wn,
                                  int left, hipStream_t s);
hipError_t launch_ext_interp(int left, const ExtDevParams &p, const int32_t *read_len, const bsw_seed_t *seeds,
                             int32_t n, const SeqPair *pairs, ExtState *st, bsw_alnreg_t *out, hipStream_t s);

}  // namespace bsw
