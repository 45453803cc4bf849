// asan_driver.cpp -- host-only driver for `make asan` (AddressSanitizer + UBSan over the host C / C++
// of the product and the oracle; no GPU).  Exercises, with result checks:
//   bsw_pack.cpp     pack_nibbles / pack_2bit on odd lengths, odd offsets, N runs, and a 9 MB
//                    buffer cut into 64-code-aligned pieces as stage_2bit cuts it; bsw_pack_batch
//                    (the 2-bit wire form) on random batches packed into exact-size heap buffers,
//                    decoded and compared, permuted / empty / N-rich batches, extents one below and
//                    at the 2^30-byte bound, cap < total_bytes and bad records rejected
//   bsw_batch.c      .bswb write / read round trip, truncated and corrupted files rejected
//   bsw_synth.c      every generator
//   bsw_ext.cpp      bsw_extend_seeds (chunked) and bsw_chain2aln through an oracle-backed engine
//                    stub (engine_stub.cpp) == oracle_extend_seeds / oracle_chain2aln, with l_pac
//   oracle/*.c       ksw_extend2, the SSE4.1 batch, ksw_align2, ksw_global2, the FM-index,
//                    mem_collect_intv and mem_chain on random inputs
// Exit status 0 = every check passed (sanitizer reports abort the run).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <vector>
#include "../../include/bsw.h"
#include "../../include/bsw_batch.h"
#include "../../include/bsw_ext.h"
#include "../../include/bsw_fmi.h"
#include "../../bwa-mem2-arm_amd/csrc/bsw_internal.h"

extern "C" {
bsw_ctx_t *stub_ctx_create(const bsw_params_t *p);
void stub_ctx_destroy(bsw_ctx_t *c);
typedef struct { uint64_t seed; int32_t tlen, qlen, h0_lo, h0_hi; double p_sub, p_indel, p_unrelated, p_n; } synth_cfg;
typedef struct { uint64_t seed; int32_t read_len, min_seed; double p_sub, p_indel, p_unrelated; } reads_cfg;
typedef struct { uint64_t seed; int32_t read_len, win_len, a, min_seed; double p_true, p_sub, p_indel; } mates_cfg;
typedef struct { uint64_t seed; int32_t read_len, w_cap, a, o_del, e_del, o_ins, e_ins; double p_sub, p_indel; } globals_cfg;
void bsw_synth_default(synth_cfg *c);
void bsw_synth_batch(const synth_cfg *c, int64_t base, int32_t n, SeqPair *pairs, uint8_t *ref, uint8_t *qer);
void bsw_synth_reference(uint64_t seed, int64_t len, double p_n, uint8_t *out);
void bsw_reads_default(reads_cfg *c);
int32_t bsw_synth_reads(const reads_cfg *c, const uint8_t *ref, int64_t ref_len, int64_t base, int32_t n, uint8_t *reads,
                        bsw_seed_t *seeds, int64_t *origin);
int32_t bsw_synth_pe_seeds(const reads_cfg *c, const uint8_t *ref, int64_t ref_len, int64_t pair_base, int32_t n_pairs,
                           int32_t ins_lo, int32_t ins_hi, double p_spurious, uint8_t *reads, bsw_seed_t *seeds,
                           int32_t *seed_read, int32_t *seed_chain);
void bsw_mates_default(mates_cfg *c);
int32_t bsw_synth_mates(const mates_cfg *c, const uint8_t *ref, int64_t ref_len, int64_t base, int32_t n,
                        SeqPair *pairs, uint8_t *qer);
void bsw_globals_default(globals_cfg *c);
int32_t bsw_synth_globals(const globals_cfg *c, const uint8_t *ref, int64_t ref_len, int64_t base, int32_t n,
                          SeqPair *pairs, uint8_t *qer);

typedef struct { int32_t o_del, e_del, o_ins, e_ins, zdrop, end_bonus; int8_t mat[25]; } oparams_t;
void oracle_get_scores(const oparams_t *p, SeqPair *pairs, const uint8_t *r, const uint8_t *q, int32_t n, int32_t w);
int sse41_get_scores16(const oparams_t *p, SeqPair *pairs, const uint8_t *ref, const uint8_t *qer, int32_t n,
                       int32_t w, int nthreads);
void oracle_extend_seeds(const oparams_t *p, const bsw_ext_opt_t *opt, const uint8_t *ref, int64_t ref_len,
                         const uint8_t *reads, const int64_t *read_off, const int32_t *read_len,
                         const bsw_seed_t *seeds, int32_t n, bsw_alnreg_t *out);
void oracle_chain2aln(const oparams_t *p, const bsw_ext_opt_t *opt, const uint8_t *ref, int64_t ref_len,
                      const uint8_t *reads, const int64_t *read_off, const int32_t *read_len, const bsw_seed_t *seeds,
                      const int32_t *seed_read, const int32_t *seed_chain, int32_t ns, bsw_alnreg_t *out,
                      int32_t *extended);
void oracle_ksw_align2_batch(const void *pairs, const uint8_t *ref, const uint8_t *qer, int n, const int8_t *mat,
                             int o_del, int e_del, int o_ins, int e_ins, void *aln, int nthreads);
void oracle_ksw_global2_batch(const void *pairs, const uint8_t *ref, const uint8_t *qer, int n, const int8_t *mat,
                              int o_del, int e_del, int o_ins, int e_ins, int32_t *score, uint32_t *cigar, int stride,
                              int32_t *n_cigar, int nthreads);
size_t oracle_fmi_sizeof(void);
int oracle_fmi_build(const uint8_t *ref, int64_t len, void *f);
void oracle_fmi_free(void *f);
void oracle_fmi_sa(const void *f, int64_t *sa);
typedef struct { int32_t min_seed_len, split_width, max_mem_intv; float split_factor; } omem_opt_t;
void oracle_collect_intv_mt(const void *f, const omem_opt_t *opt, const uint8_t *reads, const int64_t *off,
                            const int32_t *len, int32_t n, bsw_bwtintv_t *out, int32_t cap, int32_t *cnt, int nthreads);
int64_t oracle_mem_chain(const bsw_chain_opt_t *opt, const int64_t *sa, int64_t l_pac, const int32_t *read_len,
                         int32_t n_reads, const bsw_bwtintv_t *mems, int32_t cap, const int32_t *n_mems,
                         bsw_seed_t *seeds, int32_t *seed_read, int32_t *seed_chain, int64_t seed_cap);
}

static int g_fail = 0;
#define CHECK(c, ...)                                                    \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "CHECK failed %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                                \
            fprintf(stderr, "\n");                                       \
            ++g_fail;                                                    \
        }                                                                \
    } while (0)

static uint64_t g_s = 12345;
static uint32_t rnd()
{
    g_s = g_s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(g_s >> 33);
}

static void default_params(bsw_params_t *p, oparams_t *o)
{
    memset(p, 0, sizeof(*p));                          // bwa-mem defaults (bsw_params_default lives in
    p->o_del = p->o_ins = 6;                           // the HIP host file, not linked here)
    p->e_del = p->e_ins = 1;
    p->zdrop = 100;
    p->end_bonus = 5;
    p->w_match = 1; p->w_mismatch = -4; p->w_ambig = -1;
    for (int t = 0; t < 5; ++t)
        for (int q = 0; q < 5; ++q) p->mat[t * 5 + q] = (t == 4 || q == 4) ? -1 : (t == q ? 1 : -4);
    o->o_del = p->o_del; o->e_del = p->e_del; o->o_ins = p->o_ins; o->e_ins = p->e_ins;
    o->zdrop = p->zdrop; o->end_bonus = p->end_bonus;
    memcpy(o->mat, p->mat, 25);
}

static void test_pack()
{
    // odd lengths / offsets, N runs; 2-bit codes + exception words must restore the input
    for (int t = 0; t < 300; ++t) {
        const size_t n = t < 200 ? (size_t)t : (size_t)(rnd() % 20000);
        const size_t lead = rnd() % 7;
        std::vector<uint8_t> src(n + lead + 1);
        for (auto &b : src) b = rnd() % 64 ? rnd() % 4 : 4;
        const uint8_t *s = src.data() + lead;
        std::vector<uint8_t> two((n + 3) / 4 + 8, 0xcc), nib((n + 1) / 2 + 8, 0xcc);
        std::vector<uint32_t> exc;
        const uint32_t pos0 = rnd() % 1000;
        bsw::pack_2bit(two.data(), s, n, pos0, exc);
        bsw::pack_nibbles(nib.data(), s, n);
        std::vector<uint8_t> back(n);
        for (size_t k = 0; k < n; ++k) back[k] = (two[k >> 2] >> (2 * (k & 3))) & 3;
        for (uint32_t e : exc) {
            const uint32_t pos = (e >> 2) - pos0;
            CHECK(pos < n, "exception position %u out of range %zu", pos, n);
            if (pos < n) back[pos] = (uint8_t)(back[pos] | (e & 3) << 2);
        }
        CHECK(n == 0 || memcmp(back.data(), s, n) == 0, "2-bit round trip, n %zu lead %zu", n, lead);
        for (size_t k = 0; k < n; ++k) {
            const uint8_t v = (nib[k >> 1] >> (4 * (k & 1))) & 15;
            if (v != s[k]) { CHECK(false, "nibble round trip n %zu at %zu", n, k); break; }
        }
    }
    // 9 MB cut into pieces at multiples of 64 codes (stage_2bit), N on both sides of each cut
    const size_t n = 9u << 20;
    std::vector<uint8_t> src(n);
    for (size_t k = 0; k < n; ++k) src[k] = (k % 64 == 0 || k % 64 == 63) ? 4 : rnd() % 4;
    std::vector<uint8_t> two(n / 4 + 8);
    const int parts = 3;
    std::vector<uint32_t> all;
    for (int p = 0; p < parts; ++p) {
        const size_t a = (n * p / parts) & ~(size_t)63, b = p + 1 == parts ? n : (n * (p + 1) / parts) & ~(size_t)63;
        std::vector<uint32_t> exc;
        bsw::pack_2bit(two.data() + a / 4, src.data() + a, b - a, (uint32_t)a, exc);
        all.insert(all.end(), exc.begin(), exc.end());
    }
    size_t bad = 0;
    std::vector<uint8_t> back(n);
    for (size_t k = 0; k < n; ++k) back[k] = (two[k >> 2] >> (2 * (k & 3))) & 3;
    for (uint32_t e : all) back[e >> 2] = (uint8_t)(back[e >> 2] | (e & 3) << 2);
    for (size_t k = 0; k < n; ++k) bad += back[k] != src[k];
    CHECK(bad == 0 && all.size() == n / 32, "9 MB pieces: %zu wrong codes, %zu exceptions", bad, all.size());
}

// the wire form's inverse (bsw.h bsw_packed_t): records, 2-bit planes, exception words
static bool unpack_wire(const uint8_t *b, const bsw_packed_t &d, std::vector<int32_t> &rec, std::vector<uint8_t> &ref,
                        std::vector<uint8_t> &qer)
{
    rec.assign((size_t)d.n * 5, 0);
    if (d.n > 0) memcpy(rec.data(), b + d.rec_off, (size_t)d.n * 20);
    auto planes = [&](int64_t off, int64_t nb, std::vector<uint8_t> &out) {
        out.resize((size_t)nb);
        for (int64_t k = 0; k < nb; ++k) out[(size_t)k] = (b[off + k / 4] >> (2 * (k & 3))) & 3;
    };
    planes(d.ref_off, d.ref_bytes, ref);
    planes(d.qer_off, d.qer_bytes, qer);
    const uint32_t *ex = (const uint32_t *)(b + d.exc_off);
    for (int32_t k = 0; k < d.n_exc_ref + d.n_exc_qer; ++k) {
        std::vector<uint8_t> &o = k < d.n_exc_ref ? ref : qer;
        const uint32_t pos = ex[k] >> 2;
        if (pos >= o.size()) return false;
        o[pos] = (uint8_t)(o[pos] | (ex[k] & 3) << 2);
    }
    return true;
}

static void test_pack_batch()
{
    for (int it = 0; it < 60; ++it) {
        const int32_t n = it < 3 ? it : (int32_t)(rnd() % 2000);
        const bool permute = it % 4 == 3, nrich = it % 5 == 4;
        std::vector<SeqPair> pairs((size_t)n);
        std::vector<uint8_t> ref, qer;
        for (int32_t i = 0; i < n; ++i) {
            SeqPair &p = pairs[(size_t)i];
            memset(&p, 0, sizeof(p));
            p.len1 = rnd() % 9 == 0 ? 0 : (int32_t)(rnd() % 320);
            p.len2 = rnd() % 11 == 0 ? 0 : (int32_t)(rnd() % 170);
            p.h0 = (int32_t)(rnd() % 200);
            p.idr = (int32_t)ref.size() + (int32_t)(rnd() % 3);       // small gaps between windows
            p.idq = (int32_t)qer.size();
            ref.resize((size_t)p.idr + (size_t)p.len1, 0);
            qer.resize((size_t)p.idq + (size_t)p.len2, 0);
        }
        for (auto &c : ref) c = (uint8_t)(nrich && rnd() % 3 == 0 ? 4 + rnd() % 12 : rnd() % 64 ? rnd() % 4 : 4);
        for (auto &c : qer) c = (uint8_t)(nrich && rnd() % 3 == 0 ? 4 + rnd() % 12 : rnd() % 64 ? rnd() % 4 : 4);
        if (permute)
            for (int32_t i = n - 1; i > 0; --i) std::swap(pairs[(size_t)i], pairs[rnd() % (uint32_t)(i + 1)]);
        // exact-size heap copies: a read past either buffer is an ASan report
        uint8_t *r = (uint8_t *)malloc(ref.size() + 1), *q = (uint8_t *)malloc(qer.size() + 1);
        if (!ref.empty()) memcpy(r, ref.data(), ref.size());
        if (!qer.empty()) memcpy(q, qer.data(), qer.size());
        bsw_packed_t d;
        int rc = bsw_pack_batch(n ? pairs.data() : nullptr, r, q, n, nullptr, 0, &d);
        CHECK(rc == BSW_OK, "pack_batch size rc %d (n %d)", rc, n);
        uint8_t *buf = (uint8_t *)malloc((size_t)d.total_bytes + 1);
        if (d.total_bytes > 0) {
            CHECK(bsw_pack_batch(pairs.data(), r, q, n, buf, d.total_bytes - 1, &d) == BSW_E_INVAL, "cap < total");
        }
        rc = bsw_pack_batch(n ? pairs.data() : nullptr, r, q, n, buf, d.total_bytes, &d);
        CHECK(rc == BSW_OK, "pack_batch rc %d", rc);
        std::vector<int32_t> rec;
        std::vector<uint8_t> ur, uq;
        CHECK(unpack_wire(buf, d, rec, ur, uq), "exception position outside its extent");
        int64_t r_lo = INT64_MAX, q_lo = INT64_MAX;
        for (const SeqPair &p : pairs) {
            if (p.len1 > 0) r_lo = std::min<int64_t>(r_lo, p.idr);
            if (p.len2 > 0) q_lo = std::min<int64_t>(q_lo, p.idq);
        }
        size_t bad = 0;
        for (int32_t i = 0; i < n; ++i) {
            const SeqPair &p = pairs[(size_t)i];
            const int32_t *o = &rec[(size_t)i * 5];
            bad += o[2] != p.len1 || o[3] != p.len2 || o[4] != p.h0;
            for (int32_t k = 0; k < p.len1; ++k) bad += ur[(size_t)o[0] + k] != (ref[(size_t)p.idr + k] & 15);
            for (int32_t k = 0; k < p.len2; ++k) bad += uq[(size_t)o[1] + k] != (qer[(size_t)p.idq + k] & 15);
            bad += p.len1 > 0 && (int64_t)o[0] != p.idr - r_lo;
            bad += p.len2 > 0 && (int64_t)o[1] != p.idq - q_lo;
        }
        CHECK(bad == 0, "wire round trip: %zu mismatches (n %d, permute %d, nrich %d)", bad, n, permute, nrich);
        if (n > 3) {                                      // a bad record anywhere: BSW_E_RANGE
            std::vector<SeqPair> b2 = pairs;
            b2[(size_t)(rnd() % (uint32_t)n)].len2 = -1;
            CHECK(bsw_pack_batch(b2.data(), r, q, n, nullptr, 0, &d) == BSW_E_RANGE, "negative length accepted");
        }
        free(buf);
        free(r);
        free(q);
    }
    // extents one below and at the 2^30-byte bound (30-bit exception positions): the first packs and
    // round-trips its N bases at the far end, the second is BSW_E_RANGE before any byte is read
    const size_t lim = (size_t)1 << 30;
    uint8_t *big = (uint8_t *)calloc(lim + 64, 1);
    uint8_t qq[8] = {0, 1, 2, 3, 4, 0, 1, 2};
    if (big) {
        big[lim - 3] = 4;
        big[lim - 2] = 7;
        SeqPair two[2];
        memset(two, 0, sizeof(two));
        two[0].len1 = 10; two[0].idr = 0; two[0].len2 = 8; two[0].idq = 0;
        two[1].len1 = 10; two[1].idr = (int32_t)(lim - 10); two[1].len2 = 8; two[1].idq = 0;
        bsw_packed_t d;
        CHECK(bsw_pack_batch(two, big, qq, 2, nullptr, 0, &d) == BSW_E_RANGE, "extent of exactly 2^30 accepted");
        two[1].idr = (int32_t)(lim - 11);                // extent = 2^30 - 1: valid
        CHECK(bsw_pack_batch(two, big, qq, 2, nullptr, 0, &d) == BSW_OK && d.ref_bytes == (int64_t)lim - 1,
              "extent 2^30 - 1 rejected");
        uint8_t *buf = (uint8_t *)malloc((size_t)d.total_bytes);
        CHECK(buf && bsw_pack_batch(two, big, qq, 2, buf, d.total_bytes, &d) == BSW_OK, "pack at the bound");
        std::vector<int32_t> rec;
        std::vector<uint8_t> ur, uq;
        CHECK(buf && unpack_wire(buf, d, rec, ur, uq) && ur[lim - 3] == 4 && ur[lim - 2] == 7 && uq[4] == 4 &&
              d.n_exc_ref == 2 && d.n_exc_qer == 1, "exceptions at the far end of a 2^30 - 1 extent");
        free(buf);
        two[1].idr = (int32_t)(lim - 9);                 // extent = 2^30 + 1: past the bound
        CHECK(bsw_pack_batch(two, big, qq, 2, nullptr, 0, &d) == BSW_E_RANGE, "extent past 2^30 accepted");
        free(big);
    }
}

static void test_batch_file()
{
    bsw_params_t p;
    oparams_t o;
    default_params(&p, &o);
    synth_cfg c;
    bsw_synth_default(&c);
    const int n = 500;
    std::vector<SeqPair> pairs(n);
    std::vector<uint8_t> ref((size_t)n * c.tlen), qer((size_t)n * c.qlen);
    bsw_synth_batch(&c, 0, n, pairs.data(), ref.data(), qer.data());
    const char *path = "/tmp/asan_driver.bswb";
    CHECK(bswb_write(path, &p, 100, 16, 0, pairs.data(), n, ref.data(), (int64_t)ref.size(), qer.data(),
                     (int64_t)qer.size()) == BSW_OK, "bswb_write");
    bswb_header_t h;
    CHECK(bswb_read_header(path, &h) == BSW_OK, "bswb_read_header");
    std::vector<SeqPair> p2(n);
    std::vector<uint8_t> r2(ref.size()), q2(qer.size());
    CHECK(bswb_read(path, &h, p2.data(), r2.data(), q2.data()) == BSW_OK, "bswb_read");
    CHECK(memcmp(p2.data(), pairs.data(), n * sizeof(SeqPair)) == 0 && r2 == ref && q2 == qer, "round trip");
    // truncated / corrupted
    FILE *f = fopen(path, "r+b");
    fseek(f, 0, SEEK_END);
    const long len = ftell(f);
    fseek(f, len / 2, SEEK_SET);
    fputc(0x5a ^ fgetc(f), f);
    fclose(f);
    CHECK(bswb_read(path, &h, p2.data(), r2.data(), q2.data()) != BSW_OK, "corruption detected");
    CHECK(truncate(path, len - 10) == 0, "truncate");
    CHECK(bswb_read_header(path, &h) != BSW_OK || bswb_read(path, &h, p2.data(), r2.data(), q2.data()) != BSW_OK,
          "truncation detected");
    remove(path);
}

static bool same_regions(const bsw_alnreg_t *a, const bsw_alnreg_t *b, int64_t n)
{
    return memcmp(a, b, sizeof(bsw_alnreg_t) * (size_t)n) == 0;
}

static void test_extension_and_synth()
{
    bsw_params_t p;
    oparams_t o;
    default_params(&p, &o);
    bsw_ctx_t *ctx = stub_ctx_create(&p);
    const int64_t RL = 400000;
    std::vector<uint8_t> ref(RL);
    bsw_synth_reference(7, RL, 0.001, ref.data());
    reads_cfg rc;
    bsw_reads_default(&rc);
    bsw_ext_opt_t opt;
    bsw_ext_opt_default(&opt);
    {   // one seed per read (chunked by the stub's ext_chunk_cap)
        const int n = 20000;
        std::vector<uint8_t> reads((size_t)n * rc.read_len);
        std::vector<bsw_seed_t> seeds(n);
        std::vector<int64_t> origin(n), off(n);
        std::vector<int32_t> len(n, rc.read_len);
        bsw_synth_reads(&rc, ref.data(), RL, 0, n, reads.data(), seeds.data(), origin.data());
        for (int i = 0; i < n; ++i) off[i] = (int64_t)i * rc.read_len;
        std::vector<bsw_alnreg_t> got(n), want(n);
        CHECK(bsw_extend_seeds(ctx, &opt, ref.data(), RL, reads.data(), off.data(), len.data(), seeds.data(), n,
                               got.data()) == BSW_OK, "bsw_extend_seeds");
        oracle_extend_seeds(&o, &opt, ref.data(), RL, reads.data(), off.data(), len.data(), seeds.data(), n,
                            want.data());
        CHECK(same_regions(got.data(), want.data(), n), "extend_seeds == oracle");
    }
    {   // PE chains through chain2aln, on one strand and on a two-strand text (l_pac)
        const int np = 6000;
        std::vector<uint8_t> reads((size_t)2 * np * rc.read_len);
        std::vector<bsw_seed_t> seeds((size_t)2 * np * 9);
        std::vector<int32_t> sr(seeds.size()), sc(seeds.size());
        const int32_t ns = bsw_synth_pe_seeds(&rc, ref.data(), RL, 0, np, 400, 600, 0.1, reads.data(), seeds.data(),
                                              sr.data(), sc.data());
        CHECK(ns > 0, "pe seeds");
        std::vector<int64_t> off(2 * np);
        std::vector<int32_t> len(2 * np, rc.read_len);
        for (int i = 0; i < 2 * np; ++i) off[i] = (int64_t)i * rc.read_len;
        for (int pass = 0; pass < 2; ++pass) {
            std::vector<uint8_t> T = ref;
            bsw_ext_opt_t op = opt;
            if (pass == 1) {                                  // forward + reverse-complement text
                T.resize(2 * RL);
                for (int64_t i = 0; i < RL; ++i) T[2 * RL - 1 - i] = ref[i] < 4 ? 3 - ref[i] : 4;
                op.l_pac = RL;
            }
            std::vector<bsw_alnreg_t> got(ns), want(ns);
            std::vector<int32_t> ge(ns), we(ns);
            CHECK(bsw_chain2aln(ctx, &op, T.data(), (int64_t)T.size(), reads.data(), off.data(), len.data(), 2 * np,
                                seeds.data(), sr.data(), sc.data(), ns, got.data(), ge.data()) == BSW_OK,
                  "bsw_chain2aln pass %d", pass);
            oracle_chain2aln(&o, &op, T.data(), (int64_t)T.size(), reads.data(), off.data(), len.data(), seeds.data(),
                             sr.data(), sc.data(), ns, want.data(), we.data());
            CHECK(same_regions(got.data(), want.data(), ns) && ge == we, "chain2aln == oracle pass %d", pass);
        }
    }
    {   // remaining generators + the other oracles
        synth_cfg c;
        bsw_synth_default(&c);
        const int n = 3000;
        std::vector<SeqPair> pairs(n), p2;
        std::vector<uint8_t> r((size_t)n * c.tlen), q((size_t)n * c.qlen);
        bsw_synth_batch(&c, 0, n, pairs.data(), r.data(), q.data());
        p2 = pairs;
        oracle_get_scores(&o, pairs.data(), r.data(), q.data(), n, 100);
        sse41_get_scores16(&o, p2.data(), r.data(), q.data(), n, 100, 3);
        CHECK(memcmp(pairs.data(), p2.data(), sizeof(SeqPair) * n) == 0, "sse41 == scalar");
        mates_cfg mc;
        bsw_mates_default(&mc);
        std::vector<SeqPair> mp(n);
        std::vector<uint8_t> mq((size_t)n * mc.read_len);
        CHECK(bsw_synth_mates(&mc, ref.data(), RL, 0, n, mp.data(), mq.data()) >= 0, "mates");
        std::vector<int32_t> aln((size_t)n * 7);
        oracle_ksw_align2_batch(mp.data(), ref.data(), mq.data(), n, p.mat, 6, 1, 6, 1, aln.data(), 2);
        globals_cfg gc;
        bsw_globals_default(&gc);
        std::vector<SeqPair> gp(n);
        std::vector<uint8_t> gq((size_t)n * gc.read_len);
        CHECK(bsw_synth_globals(&gc, ref.data(), RL, 0, n, gp.data(), gq.data()) >= 0, "globals");
        std::vector<int32_t> sc(n), ncig(n);
        std::vector<uint32_t> cig((size_t)n * 64);
        oracle_ksw_global2_batch(gp.data(), ref.data(), gq.data(), n, p.mat, 6, 1, 6, 1, sc.data(), cig.data(), 64,
                                 ncig.data(), 2);
    }
    {   // FM-index, intervals, chains
        const int64_t L = 50000;
        std::vector<uint8_t> r(L);
        for (auto &b : r) b = rnd() % 4;
        for (int k = 0; k < 20; ++k) memcpy(&r[1000 + k * 2000], &r[100], 300);     // dispersed repeats
        std::vector<uint8_t> fbuf(oracle_fmi_sizeof());
        CHECK(oracle_fmi_build(r.data(), L, fbuf.data()) == 0, "fmi build");
        const int n = 400, RLn = 151;
        std::vector<uint8_t> reads((size_t)n * RLn);
        std::vector<int64_t> off(n);
        std::vector<int32_t> len(n, RLn);
        for (int i = 0; i < n; ++i) {
            off[i] = (int64_t)i * RLn;
            const int64_t st = rnd() % (L - RLn);
            for (int k = 0; k < RLn; ++k) reads[off[i] + k] = rnd() % 50 ? r[st + k] : rnd() % 5;
        }
        const int cap = 512;
        std::vector<bsw_bwtintv_t> mems((size_t)n * cap);
        std::vector<int32_t> cnt(n);
        omem_opt_t mo = {19, 10, 20, 1.5f};
        oracle_collect_intv_mt(fbuf.data(), &mo, reads.data(), off.data(), len.data(), n, mems.data(), cap, cnt.data(), 2);
        std::vector<int64_t> sa(2 * L + 1);
        oracle_fmi_sa(fbuf.data(), sa.data());
        bsw_chain_opt_t co = {500, 100, 10000, 0, 19, 1 << 30, 0.5f, 0.5f};
        const int64_t need = oracle_mem_chain(&co, sa.data(), L, len.data(), n, mems.data(), cap, cnt.data(), nullptr,
                                              nullptr, nullptr, 0);
        std::vector<bsw_seed_t> s(need + 1);
        std::vector<int32_t> a(need + 1), b(need + 1);
        CHECK(oracle_mem_chain(&co, sa.data(), L, len.data(), n, mems.data(), cap, cnt.data(), s.data(), a.data(),
                               b.data(), need) == need, "mem_chain count");
        oracle_fmi_free(fbuf.data());
    }
    stub_ctx_destroy(ctx);
}

int main()
{
    test_pack();
    test_pack_batch();
    test_batch_file();
    test_extension_and_synth();
    printf("asan_driver: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
    return g_fail ? 1 : 0;
}
