// bsw_pack.cpp -- host-side code packing of the bsw_get_scores staging pipeline (bsw_host.cpp):
// nibbles and 2-bit codes + exception words, written into the pinned staging buffer with
// streaming stores.  Plain C++ (g++), so the AVX2 form can be selected at run time without the
// HIP device pass seeing x86 target attributes.
#include <emmintrin.h>
#include <immintrin.h>
#include <cstdint>
#include <cstddef>
#include <algorithm>
#include <cstring>
#include <vector>
#include "bsw_internal.h"

namespace bsw {

// 4-bit packing of base codes for the host -> device copy: staged byte k = code[2k] |
// code[2k+1] << 4 (codes 0..4 in the ABI; the low nibble of any code is kept).  Halves the
// PCIe bytes of the sequences; unpack_kernel restores the byte-per-base buffers in HBM.
void pack_nibbles(uint8_t *dst, const uint8_t *src, size_t nbytes)
{
    size_t i = 0;
    const __m128i m0 = _mm_set1_epi16(0x000f), m1 = _mm_set1_epi16(0x00f0);
    // streaming (non-temporal) stores into the pinned staging buffer when it is 16-B aligned: no
    // read-for-ownership of destination lines the CPU never reads again (the DMA engine does)
    if (((uintptr_t)dst & 15) == 0) {
        for (; i + 32 <= nbytes; i += 32) {
            const __m128i a = _mm_loadu_si128((const __m128i *)(src + i));
            const __m128i b = _mm_loadu_si128((const __m128i *)(src + i + 16));
            const __m128i ra = _mm_or_si128(_mm_and_si128(a, m0), _mm_and_si128(_mm_srli_epi16(a, 4), m1));
            const __m128i rb = _mm_or_si128(_mm_and_si128(b, m0), _mm_and_si128(_mm_srli_epi16(b, 4), m1));
            _mm_stream_si128((__m128i *)(dst + i / 2), _mm_packus_epi16(ra, rb));
        }
        _mm_sfence();
    }
    for (; i + 32 <= nbytes; i += 32) {
        const __m128i a = _mm_loadu_si128((const __m128i *)(src + i));
        const __m128i b = _mm_loadu_si128((const __m128i *)(src + i + 16));
        const __m128i ra = _mm_or_si128(_mm_and_si128(a, m0), _mm_and_si128(_mm_srli_epi16(a, 4), m1));
        const __m128i rb = _mm_or_si128(_mm_and_si128(b, m0), _mm_and_si128(_mm_srli_epi16(b, 4), m1));
        _mm_storeu_si128((__m128i *)(dst + i / 2), _mm_packus_epi16(ra, rb));
    }
    for (; i < nbytes; i += 2)
        dst[i / 2] = (uint8_t)((src[i] & 15) | (i + 1 < nbytes ? (src[i + 1] & 15) << 4 : 0));
}

// 2-bit packing (round 2): staged byte k = code[4k] | code[4k+1] << 2 | code[4k+2] << 4 |
// code[4k+3] << 6 (low two bits), plus an exception word for every byte outside 0..3 (N bases:
// 0.1% on C2), patched in HBM after the 2-bit unpack -- the same bytes in HBM as the nibble path,
// at a quarter of the byte-per-base PCIe traffic.  Exception word (round 6) = pos << 2 | bits 2-3
// of the code: the low two bits are already in the 2-bit plane, so positions get 30 bits (extents
// up to 1 GiB; 28 bits with the whole nibble in the word).
static inline uint32_t exc_word(uint32_t pos, uint8_t code) { return (pos << 2) | ((code & 15u) >> 2); }

static inline __m128i pack2_lanes(__m128i x)      // 4 codes per dword -> one byte (low byte)
{
    x = _mm_and_si128(x, _mm_set1_epi8(3));
    x = _mm_or_si128(x, _mm_srli_epi32(x, 6));     // bits 0-3: c0 | c1 << 2; bits 16-19: c2 | c3 << 2
    x = _mm_or_si128(x, _mm_srli_epi32(x, 12));    // bits 4-7: c2 | c3 << 2
    return _mm_and_si128(x, _mm_set1_epi32(0xff));
}

static void pack_2bit_sse2(uint8_t *dst, const uint8_t *src, size_t nbytes, uint32_t pos0, std::vector<uint32_t> &exc)
{
    auto scan = [&](size_t a, size_t b) {
        for (size_t k = a; k < b; ++k)
            if (src[k] & 0xfc) exc.push_back(exc_word(pos0 + (uint32_t)k, src[k]));
    };
    const __m128i hi = _mm_set1_epi8((char)0xfc), z = _mm_setzero_si128();
    const bool nt = ((uintptr_t)dst & 15) == 0;      // streaming stores (see pack_nibbles)
    size_t i = 0;
    for (; i + 64 <= nbytes; i += 64) {
        const __m128i a = _mm_loadu_si128((const __m128i *)(src + i));
        const __m128i b = _mm_loadu_si128((const __m128i *)(src + i + 16));
        const __m128i c = _mm_loadu_si128((const __m128i *)(src + i + 32));
        const __m128i d = _mm_loadu_si128((const __m128i *)(src + i + 48));
        const __m128i o = _mm_or_si128(_mm_or_si128(a, b), _mm_or_si128(c, d));
        if (_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_and_si128(o, hi), z)) != 0xffff) scan(i, i + 64);
        const __m128i r = _mm_packus_epi16(_mm_packs_epi32(pack2_lanes(a), pack2_lanes(b)),
                                           _mm_packs_epi32(pack2_lanes(c), pack2_lanes(d)));
        if (nt) _mm_stream_si128((__m128i *)(dst + i / 4), r);
        else _mm_storeu_si128((__m128i *)(dst + i / 4), r);
    }
    if (nt) _mm_sfence();
    scan(i, nbytes);
    for (; i < nbytes; i += 4) {
        uint32_t v = 0;
        for (size_t k = 0; k < 4 && i + k < nbytes; ++k) v |= (uint32_t)(src[i + k] & 3u) << (2 * k);
        dst[i / 4] = (uint8_t)v;
    }
}


// AVX2 form: 128 codes -> 32 bytes per step.  Codes are masked to 2 bits and each dword's four
// codes multiplied into its top byte: x * (2^24 + 2^18 + 2^12 + 2^6) puts c0 | c1 << 2 |
// c2 << 4 | c3 << 6 in bits 24..31 (the cross terms stay below 2^24, no carry).  Exceptions come
// from a per-vector byte mask (one bit per non-ACGT byte), visited bit by bit.
__attribute__((target("avx2"))) static inline void exc_avx2(__m256i v, const uint8_t *src, size_t at, uint32_t pos0,
                                                           std::vector<uint32_t> &exc)
{
    uint32_t m = ~(uint32_t)_mm256_movemask_epi8(
        _mm256_cmpeq_epi8(_mm256_and_si256(v, _mm256_set1_epi8((char)0xfc)), _mm256_setzero_si256()));
    while (m) {
        const size_t k = at + (size_t)__builtin_ctz(m);
        exc.push_back(exc_word(pos0 + (uint32_t)k, src[k]));
        m &= m - 1;
    }
}

__attribute__((target("avx2"))) static void pack_2bit_avx2(uint8_t *dst, const uint8_t *src, size_t nbytes,
                                                          uint32_t pos0, std::vector<uint32_t> &exc)
{
    const __m256i m3 = _mm256_set1_epi8(3), hi = _mm256_set1_epi8((char)0xfc);
    const __m256i mul = _mm256_set1_epi32(0x01041040);
    const __m256i perm = _mm256_setr_epi32(0, 4, 1, 5, 2, 6, 3, 7);
    const bool nt = ((uintptr_t)dst & 31) == 0;
    size_t i = 0;
    for (; i + 128 <= nbytes; i += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i *)(src + i));
        __m256i b = _mm256_loadu_si256((const __m256i *)(src + i + 32));
        __m256i c = _mm256_loadu_si256((const __m256i *)(src + i + 64));
        __m256i d = _mm256_loadu_si256((const __m256i *)(src + i + 96));
        const __m256i o = _mm256_or_si256(_mm256_or_si256(a, b), _mm256_or_si256(c, d));
        if (!_mm256_testz_si256(o, hi)) {
            exc_avx2(a, src, i, pos0, exc); exc_avx2(b, src, i + 32, pos0, exc);
            exc_avx2(c, src, i + 64, pos0, exc); exc_avx2(d, src, i + 96, pos0, exc);
        }
        a = _mm256_srli_epi32(_mm256_mullo_epi32(_mm256_and_si256(a, m3), mul), 24);
        b = _mm256_srli_epi32(_mm256_mullo_epi32(_mm256_and_si256(b, m3), mul), 24);
        c = _mm256_srli_epi32(_mm256_mullo_epi32(_mm256_and_si256(c, m3), mul), 24);
        d = _mm256_srli_epi32(_mm256_mullo_epi32(_mm256_and_si256(d, m3), mul), 24);
        // per 128-bit half: [a b c d] dwords of half 0, then of half 1 -> a0 a1 b0 b1 c0 c1 d0 d1
        const __m256i r = _mm256_permutevar8x32_epi32(
            _mm256_packus_epi16(_mm256_packus_epi32(a, b), _mm256_packus_epi32(c, d)), perm);
        if (nt) _mm256_stream_si256((__m256i *)(dst + i / 4), r);
        else _mm256_storeu_si256((__m256i *)(dst + i / 4), r);
    }
    if (nt) _mm_sfence();
    if (i < nbytes) pack_2bit_sse2(dst + i / 4, src + i, nbytes - i, pos0 + (uint32_t)i, exc);
}

void pack_2bit(uint8_t *dst, const uint8_t *src, size_t nbytes, uint32_t pos0, std::vector<uint32_t> &exc)
{
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) pack_2bit_avx2(dst, src, nbytes, pos0, exc);
    else pack_2bit_sse2(dst, src, nbytes, pos0, exc);
}

// seed identities (plan_kernel's seed_matches, bsw_host.cpp): best over shifts s = 0..12 of the
// matches of query[10, 40) with target[4 + s, 34 + s); 31 when the pair is too short to test
static int seed_matches_scalar(const uint8_t *q, int qlen, const uint8_t *r, int tlen)
{
    if (qlen < 40 || tlen < 46) return 31;
    int best = 0;
    for (int s = 0; s <= 12; ++s) {
        int c = 0;
        for (int j = 0; j < 30; ++j) c += q[10 + j] == r[4 + j + s];
        best = c > best ? c : best;
    }
    return best;
}

// AVX2: the 30 query bytes in one register, each shift one unaligned load + compare + popcount.
// Reads target bytes [4, 48): only when tlen >= 48 (the scalar form otherwise)
__attribute__((target("avx2,popcnt"))) static int seed_matches_avx2(const uint8_t *q, int qlen, const uint8_t *r,
                                                                    int tlen)
{
    if (qlen < 42 || tlen < 48) return seed_matches_scalar(q, qlen, r, tlen);
    const __m256i qv = _mm256_loadu_si256((const __m256i *)(q + 10));
    int best = 0;
    for (int s = 0; s <= 12; ++s) {
        const __m256i rv = _mm256_loadu_si256((const __m256i *)(r + 4 + s));
        const uint32_t m = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(qv, rv)) & 0x3fffffffu;
        const int c = __builtin_popcount(m);
        best = c > best ? c : best;
    }
    return best;
}

void fast_keys(const SeqPair *pairs, int32_t n, const uint8_t *ref, const uint8_t *qer, uint32_t *keys)
{
    static const bool avx2 = __builtin_cpu_supports("avx2");
    for (int32_t i = 0; i < n; ++i) {
        const SeqPair &p = pairs[i];
        const int qlen = p.len2 > 0 ? p.len2 : 0, tlen = p.len1 > 0 ? p.len1 : 0;
        const uint8_t *q = qer + (qlen > 0 ? p.idq : 0), *r = ref + (tlen > 0 ? p.idr : 0);
        const int mt = avx2 ? seed_matches_avx2(q, qlen, r, tlen) : seed_matches_scalar(q, qlen, r, tlen);
        const int rel = mt > 18;
        const int h0 = p.h0 < 0 ? 0 : (p.h0 > 255 ? 255 : p.h0);
        keys[i] = ((uint32_t)(255 - (qlen < 255 ? qlen : 255)) << 20) | ((uint32_t)(1 - rel) << 19) |
                  ((uint32_t)(63 - ((tlen >> 5) < 63 ? (tlen >> 5) : 63)) << 13) |
                  ((uint32_t)(31 - (mt < 31 ? mt : 31)) << 8) | (uint32_t)(255 - h0);
    }
}

__attribute__((target("bmi2"))) static void compact_bmi2(const uint32_t *keys, int32_t a0, int32_t a1, uint32_t vary,
                                                         uint64_t *kv)
{
    for (int32_t i = a0; i < a1; ++i) kv[i] = ((uint64_t)_pext_u32(keys[i], vary) << 32) | (uint32_t)i;
}

void compact_keys(const uint32_t *keys, int32_t a0, int32_t a1, uint32_t vary, uint64_t *kv)
{
    static const bool bmi2 = __builtin_cpu_supports("bmi2");
    if (bmi2) { compact_bmi2(keys, a0, a1, vary, kv); return; }
    for (int32_t i = a0; i < a1; ++i) {
        uint32_t ck = 0;
        for (uint32_t v = vary, o = 0; v; v &= v - 1, ++o) ck |= ((keys[i] >> __builtin_ctz(v)) & 1u) << o;
        kv[i] = ((uint64_t)ck << 32) | (uint32_t)i;
    }
}

}  // namespace bsw

// bsw_pack_batch (bsw.h): the 2-bit wire form of a batch, host-only
extern "C" int bsw_pack_batch(const SeqPair *pairs, const uint8_t *ref, const uint8_t *qer, int32_t n, void *dst,
                              int64_t cap, bsw_packed_t *desc)
{
    if (!desc || n < 0 || (n > 0 && !pairs) || cap < 0) return BSW_E_INVAL;
    int64_t r_lo = INT64_MAX, r_hi = 0, q_lo = INT64_MAX, q_hi = 0;
    for (int32_t i = 0; i < n; ++i) {
        const SeqPair &p = pairs[i];
        if (p.len1 < 0 || p.len2 < 0 || p.len1 > BSW_MAX_LEN || p.len2 > BSW_MAX_LEN || p.idr < 0 || p.idq < 0)
            return BSW_E_RANGE;
        if (p.len1 > 0) { r_lo = std::min<int64_t>(r_lo, p.idr); r_hi = std::max<int64_t>(r_hi, (int64_t)p.idr + p.len1); }
        if (p.len2 > 0) { q_lo = std::min<int64_t>(q_lo, p.idq); q_hi = std::max<int64_t>(q_hi, (int64_t)p.idq + p.len2); }
    }
    if (r_lo == INT64_MAX) r_lo = r_hi = 0;
    if (q_lo == INT64_MAX) q_lo = q_hi = 0;
    const int64_t rb = r_hi - r_lo, qb = q_hi - q_lo;
    if (rb >= ((int64_t)1 << 30) || qb >= ((int64_t)1 << 30)) return BSW_E_RANGE;
    if ((rb > 0 && !ref) || (qb > 0 && !qer)) return BSW_E_INVAL;
    auto count_exc = [](const uint8_t *s, int64_t len) {
        int64_t c = 0;
        for (int64_t k = 0; k < len; ++k) c += (s[k] & 0xfc) != 0;
        return c;
    };
    const int64_t er = count_exc(ref + r_lo, rb), eq = count_exc(qer + q_lo, qb);
    auto a256 = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
    bsw_packed_t d{};
    d.n = n;
    d.n_exc_ref = (int32_t)er;
    d.n_exc_qer = (int32_t)eq;
    d.ref_bytes = rb;
    d.qer_bytes = qb;
    d.rec_off = 0;
    d.ref_off = a256((int64_t)n * 20);
    d.qer_off = a256(d.ref_off + (rb + 3) / 4 + 4);
    d.exc_off = a256(d.qer_off + (qb + 3) / 4 + 4);
    d.total_bytes = a256(d.exc_off + 4 * (er + eq));
    *desc = d;
    if (!dst) return BSW_OK;
    if (cap < d.total_bytes) return BSW_E_INVAL;
    uint8_t *h = (uint8_t *)dst;
    int32_t *rec = (int32_t *)(h + d.rec_off);
    for (int32_t i = 0; i < n; ++i) {
        const SeqPair &p = pairs[i];
        rec[5 * (int64_t)i + 0] = p.len1 > 0 ? (int32_t)(p.idr - r_lo) : 0;
        rec[5 * (int64_t)i + 1] = p.len2 > 0 ? (int32_t)(p.idq - q_lo) : 0;
        rec[5 * (int64_t)i + 2] = p.len1;
        rec[5 * (int64_t)i + 3] = p.len2;
        rec[5 * (int64_t)i + 4] = p.h0;
    }
    std::vector<uint32_t> exr, exq;
    memset(h + d.ref_off, 0, (size_t)(d.qer_off - d.ref_off));
    memset(h + d.qer_off, 0, (size_t)(d.exc_off - d.qer_off));
    bsw::pack_2bit(h + d.ref_off, ref + r_lo, (size_t)rb, 0u, exr);
    bsw::pack_2bit(h + d.qer_off, qer + q_lo, (size_t)qb, 0u, exq);
    if ((int64_t)exr.size() != er || (int64_t)exq.size() != eq) return BSW_E_INVAL;   // (cannot happen)
    uint32_t *ex = (uint32_t *)(h + d.exc_off);
    if (er) memcpy(ex, exr.data(), 4 * (size_t)er);
    if (eq) memcpy(ex + er, exq.data(), 4 * (size_t)eq);
    memset(h + d.exc_off + 4 * (er + eq), 0, (size_t)(d.total_bytes - d.exc_off - 4 * (er + eq)));
    return BSW_OK;
}
