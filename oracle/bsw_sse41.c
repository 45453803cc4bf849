/*
 * oracle/bsw_sse41.c -- CPU BASELINE (test / bench infrastructure only).
 *
 * A restatement of the reference's CPU path for this hot loop: upstream bwa-mem2
 * `BandedPairWiseSW::getScores16` -> `smithWatermanBatchWrapper16` ->
 * `smithWaterman128_16` (SSE2/SSE4.1 section of src/bandedSWA.cpp, lines 3361-4872 per
 * docs-archive/ARM-BATCHED-SAM-PLAN.md:60-64), whose design the reference documents:
 *   - sort pairs by length, pad to a multiple of the SIMD width with len=0 pairs
 *     (docs-archive/WEEK1_WRAPPER_COMPLETE.md:55-58, docs-archive/WEEK2_STATUS.md:44-60);
 *   - one pair per SIMD lane, 8 x int16 lanes for the 16-bit path
 *     (docs-archive/ARM-BATCHED-SAM-PLAN.md:129-134);
 *   - AoS -> SoA transpose of both sequences with DUMMY padding
 *     (docs-archive/WEEK1_WRAPPER_COMPLETE.md:64-83);
 *   - boundary rows from h0 and per-lane band min(w, max_ins, max_del)
 *     (docs-archive/WEEK1_WRAPPER_COMPLETE.md:85-118);
 *   - threads over batches (`omp for schedule(dynamic, 128)` upstream; pthreads here).
 * The upstream C++ is not available, so this is NOT the upstream binary:
 * it is the same design, written here, and it must reproduce the scalar oracle
 * (oracle/ksw_ext_ref.c) bit for bit -- tests/test_oracle.py checks that.  Per-lane
 * semantics follow SURVEY.md Appendix A with two exact simplifications proved in
 * the left band edge is max(0, i-w) (A.9 (ii)) and the right edge after a
 * row is min(lastH + 3, qlen), lastH = last column with H(i,j) > 0.
 *
 * bench.py reports it as cpu_baseline kind "port".
 */
#include <smmintrin.h>
#include "bsw_simd_common.h"

/* SSE4.1: 8 x int16 lanes, compare results as all-ones vectors */
#define W16 8
#define SIMD_NAME(x) sse_##x
#define SIMD_FN
#define SIMD_ENTRY sse41_get_scores16
typedef __m128i VEC;
typedef __m128i MASK;
#define V_SET1(x) _mm_set1_epi16((short)(x))
#define V_LOADU(p) _mm_loadu_si128((const __m128i *)(p))
#define V_STOREU(p, v) _mm_storeu_si128((__m128i *)(p), (v))
#define V_ADD _mm_add_epi16
#define V_SUB _mm_sub_epi16
#define V_MAX _mm_max_epi16
#define V_CMPEQ _mm_cmpeq_epi16
#define V_CMPGT _mm_cmpgt_epi16
#define V_CMPLT _mm_cmplt_epi16
#define V_BLEND(a, b, m) _mm_blendv_epi8((a), (b), (m))
#define V_ZERO_WHERE(m, v) _mm_andnot_si128((m), (v))
#define M_AND _mm_and_si128
#define M_OR _mm_or_si128
#define M_FROM_V(v) (v)

#include "bsw_simd_batch.inc"
