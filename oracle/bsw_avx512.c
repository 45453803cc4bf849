/*
 * oracle/bsw_avx512.c -- CPU BASELINE context legs (test / bench infrastructure only).
 *
 * The same restatement as oracle/bsw_sse41.c (upstream's getScores16 batch design, one pair per
 * SIMD lane), at the widths upstream bwa-mem2 v2.2.1 dispatches on hosts that have them:
 * smithWaterman256_16 (AVX2, 16 x int16 lanes: bandedSWA.cpp's AVX2 section, lines 263-1817) and
 * smithWaterman512_16 (AVX-512BW, 32 x int16 lanes: lines 1818-3360; section boundaries per
 * docs-archive/ARM-BATCHED-SAM-PLAN.md:60-71, SIMD widths per :129-134).  north_star names the
 * SSE4.1 / scalar path as the baseline, so bench.py keeps SSE4.1 as cpu_baseline.value and
 * reports these beside it: what the same upstream binary would run on a Zen 5 / Xeon host.
 * Functions carry their own target attributes; callers check the CPU (avx2_supported /
 * avx512bw_supported) first.  Bit-exact against the scalar oracle (tests/test_oracle.py).
 */
#include <immintrin.h>
#include "bsw_simd_common.h"

int avx2_supported(void) { return __builtin_cpu_supports("avx2"); }
int avx512bw_supported(void) { return __builtin_cpu_supports("avx512bw"); }

/* ---- AVX-512BW: 32 x int16 lanes, compare results in k-mask registers */
#pragma GCC push_options
#pragma GCC target("avx512f,avx512bw")
#define W16 32
#define SIMD_NAME(x) avx512_##x
#define SIMD_FN __attribute__((target("avx512f,avx512bw")))
#define SIMD_ENTRY avx512_get_scores16
typedef __m512i VEC;
typedef __mmask32 MASK;
#define V_SET1(x) _mm512_set1_epi16((short)(x))
#define V_LOADU(p) _mm512_loadu_si512((const void *)(p))
#define V_STOREU(p, v) _mm512_storeu_si512((void *)(p), (v))
#define V_ADD _mm512_add_epi16
#define V_SUB _mm512_sub_epi16
#define V_MAX _mm512_max_epi16
#define V_CMPEQ _mm512_cmpeq_epi16_mask
#define V_CMPGT _mm512_cmpgt_epi16_mask
#define V_CMPLT _mm512_cmplt_epi16_mask
#define V_BLEND(a, b, m) _mm512_mask_blend_epi16((m), (a), (b))
#define V_ZERO_WHERE(m, v) _mm512_maskz_mov_epi16((__mmask32)~(m), (v))
#define M_AND(a, b) ((MASK)((a) & (b)))
#define M_OR(a, b) ((MASK)((a) | (b)))
#define M_FROM_V(v) _mm512_cmpneq_epi16_mask((v), _mm512_setzero_si512())
#include "bsw_simd_batch.inc"
#undef W16
#undef SIMD_NAME
#undef SIMD_FN
#undef SIMD_ENTRY
#undef V_SET1
#undef V_LOADU
#undef V_STOREU
#undef V_ADD
#undef V_SUB
#undef V_MAX
#undef V_CMPEQ
#undef V_CMPGT
#undef V_CMPLT
#undef V_BLEND
#undef V_ZERO_WHERE
#undef M_AND
#undef M_OR
#undef M_FROM_V
#pragma GCC pop_options

/* ---- AVX2: 16 x int16 lanes, compare results as all-ones vectors */
#pragma GCC push_options
#pragma GCC target("avx2")
#define W16 16
#define SIMD_NAME(x) avx2_##x
#define SIMD_FN __attribute__((target("avx2")))
#define SIMD_ENTRY avx2_get_scores16
#define VEC __m256i
#define MASK __m256i
#define V_SET1(x) _mm256_set1_epi16((short)(x))
#define V_LOADU(p) _mm256_loadu_si256((const __m256i *)(p))
#define V_STOREU(p, v) _mm256_storeu_si256((__m256i *)(p), (v))
#define V_ADD _mm256_add_epi16
#define V_SUB _mm256_sub_epi16
#define V_MAX _mm256_max_epi16
#define V_CMPEQ _mm256_cmpeq_epi16
#define V_CMPGT _mm256_cmpgt_epi16
#define V_CMPLT(a, b) _mm256_cmpgt_epi16((b), (a))
#define V_BLEND(a, b, m) _mm256_blendv_epi8((a), (b), (m))
#define V_ZERO_WHERE(m, v) _mm256_andnot_si256((m), (v))
#define M_AND _mm256_and_si256
#define M_OR _mm256_or_si256
#define M_FROM_V(v) (v)
#include "bsw_simd_batch.inc"
#pragma GCC pop_options
