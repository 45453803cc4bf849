// bsw_fmi.hip -- FM-index SMEM seeding on gfx950 (include/bsw_fmi.h).
//
// Index (host build, resident in HBM):
//   T = ref + revcomp(ref), n = |T|; rows r = 0..n of the sorted suffixes of T$ (row 0 = '$').
//   Suffix array by prefix doubling: one 64-bit LSD radix sort of 27-base keys (base 5 with
//   '$'/past-the-end = 0, so suffixes that reach '$' inside the key are already unique), then
//   only the remaining tie groups are re-sorted by rank[i + h], h = 27, 54, 108, ... (ranks =
//   group starts, refined in place).
//   Occ blocks: one 64-byte block per 64 BWT rows -- cnt[c] = #c in rows [0, 64b) (uint32) and
//   bits[c] = one-hot mask of rows 64b + y holding c (bit y) -- so Occ(c, r) = cnt[c] +
//   popcount(bits[c] & ((1 << (r & 63)) - 1)) is ONE 64-byte load (bwa-mem2's CP_OCC layout with
//   32-bit counts).  The '$' row has no bit set.
//
// Kernel (one lane per read; the FM-index walk is a serial chain of dependent, data-dependent
// HBM loads, so the GPU's job is to keep ~10^5 such chains in flight, not to vectorise one):
//   backward extension of (k, l, s) by base a (FMI_search::backwardExt):
//     k' = count[a] + Occ(a, k), s' = Occ(a, k + s) - Occ(a, k),
//     l' = l + [k <= sentinel < k + s] + sum_{b > a} (Occ(b, k + s) - Occ(b, k))
//   forward extension by read base q = backward extension of the swapped interval (l, k, s) by
//   3 - q, swapped back.  Rows k and k + s share one block whenever s is small (the common
//   case after a few bases), and then one load serves both.
//   bwt_smem1a / bwt_seed_strategy1 / mem_collect_intv control flow as in oracle/fmi_ref.c;
//   the per-read interval vectors (prev / curr) live in HBM scratch laid out [slot][read] (16 B
//   per entry: k, l, s, end), the output intervals at mems[read * cap + t], sorted in place
//   by an insertion sort at the end.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>
#include "../../include/bsw_fmi.h"
#include "bsw_fmi_internal.h"

namespace {

using bsw::FmiBlock;
using bsw::FmiBlockW;

template <class U>
struct FmiDevT {                     // kernel view of the resident index (U = row / count width)
    const void *blk;
    U count[5];
    U sentinel;
    U n;                             // |T|
    // text mode (null when built with BSW_FMI_NO_TEXT): T with 0xFF padding past n, SA, SA^-1
    const uint8_t *text;
    const U *sa;
    const U *isa;
    // k-mer interval table (null / kt = 0: off): the exact (k, l, s) of every string of 1 .. kt
    // bases, level j at ktab + (4^j - 4) / 3, code = the bases as a base-4 number (first base most
    // significant); 16 B per entry (ktab_get)
    const uint4 *ktab;
    int kt;
    // the same levels' counts s alone, 4 B per entry (null: off) -- the sweeps' virtual entries
    // need only s, and a level's 4-B form is 4x denser in the caches (levels <= 12 of a 3 Gb
    // genome: 89 MB)
    const uint32_t *stab;
};

// text-mode interval entries keep the occurrence's text position in k; their end carries this
// flag (k, l are resolved through SA^-1 only when the interval is output)
constexpr uint32_t kTextFlag = 0x80000000u;

// backward sweep: stored entries extended together.  1 since the virtual entries: the stored part of a
// vector is mostly one or two long entries, and a batch pads with duplicate extensions of its last entry
// (random block loads for nothing): C4 at 3 Gb 221.5 -> 208.0 ms per step at 1, 264.7 at 3
// (profiles/r05/smem_virtual_entries_ab.txt)
#ifndef BSW_SMEM_BACK_UNROLL
#define BSW_SMEM_BACK_UNROLL 1
#endif
constexpr int kBackUnroll = BSW_SMEM_BACK_UNROLL;
#ifndef BSW_SMEM_VIRT_UNROLL
#define BSW_SMEM_VIRT_UNROLL 2
#endif
constexpr int kVirtUnroll = BSW_SMEM_VIRT_UNROLL;   // the same for the virtual entries' table loads

struct MemOpt {
    int32_t min_seed_len, split_width, max_mem_intv, split_len;
};

// ---------------------------------------------------------------- device: index queries

template <class U>
struct Occ4 {                        // one block: the running counts and the four masks
    U c[4];
    uint64_t b[4];
};

__device__ __forceinline__ void load_block(const void *blk, uint32_t bi, Occ4<uint32_t> &o)
{
    const FmiBlock *b = (const FmiBlock *)blk + bi;
    const uint4 cnt = *reinterpret_cast<const uint4 *>(b);
    const ulonglong2 b01 = reinterpret_cast<const ulonglong2 *>(b)[2];
    const ulonglong2 b23 = reinterpret_cast<const ulonglong2 *>(b)[3];
    o.c[0] = cnt.x; o.c[1] = cnt.y; o.c[2] = cnt.z; o.c[3] = cnt.w;
    o.b[0] = b01.x; o.b[1] = b01.y; o.b[2] = b23.x; o.b[3] = b23.y;
}
__device__ __forceinline__ void load_block(const void *blk, uint64_t bi, Occ4<uint64_t> &o)
{
    const FmiBlockW *b = (const FmiBlockW *)blk + bi;
    const ulonglong2 c01 = reinterpret_cast<const ulonglong2 *>(b)[0];
    const ulonglong2 c23 = reinterpret_cast<const ulonglong2 *>(b)[1];
    const ulonglong2 b01 = reinterpret_cast<const ulonglong2 *>(b)[2];
    const ulonglong2 b23 = reinterpret_cast<const ulonglong2 *>(b)[3];
    o.c[0] = c01.x; o.c[1] = c01.y; o.c[2] = c23.x; o.c[3] = c23.y;
    o.b[0] = b01.x; o.b[1] = b01.y; o.b[2] = b23.x; o.b[3] = b23.y;
}

template <class U>
__device__ __forceinline__ U occ_of(const Occ4<U> &o, int c, uint64_t mask)
{
    const U cc = c == 0 ? o.c[0] : c == 1 ? o.c[1] : c == 2 ? o.c[2] : o.c[3];
    const uint64_t bb = c == 0 ? o.b[0] : c == 1 ? o.b[1] : c == 2 ? o.b[2] : o.b[3];
    return cc + (U)__builtin_popcountll(bb & mask);
}

template <class U>
struct IvT {
    U k, l, s;
};

// FMI_search::backwardExt restricted to the one base the caller keeps
template <class U>
__device__ __forceinline__ IvT<U> backward_ext(const FmiDevT<U> &f, IvT<U> in, int a)
{
    const U sp = in.k, ep = in.k + in.s;
    if (ep > f.n + 1 || ep < sp) return IvT<U>{0, 0, 0};   // never for a consistent index (bsw_fmi_check)
    Occ4<U> o0, o1;
    load_block(f.blk, sp >> 6, o0);
    if ((ep >> 6) == (sp >> 6)) o1 = o0;
    else load_block(f.blk, ep >> 6, o1);
    const uint64_t ms = (sp & 63) ? (~0ull >> (64 - (sp & 63))) : 0ull;
    const uint64_t me = (ep & 63) ? (~0ull >> (64 - (ep & 63))) : 0ull;
    U osp[4], oep[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        osp[b] = occ_of(o0, b, ms);
        oep[b] = occ_of(o1, b, me);
    }
    U l = in.l + ((sp <= f.sentinel && ep > f.sentinel) ? (U)1 : (U)0);
    // l[3] = l + sent; l[b] = l[b + 1] + s[b + 1]
#pragma unroll
    for (int b = 3; b > 0; --b)
        if (b > a) l += oep[b] - osp[b];
    IvT<U> o;
    const U ca = a == 0 ? f.count[0] : a == 1 ? f.count[1] : a == 2 ? f.count[2] : f.count[3];
    const U oa = a == 0 ? osp[0] : a == 1 ? osp[1] : a == 2 ? osp[2] : osp[3];
    const U ea = a == 0 ? oep[0] : a == 1 ? oep[1] : a == 2 ? oep[2] : oep[3];
    o.k = ca + oa;
    o.s = ea - oa;
    o.l = l;
    return o;
}

template <class U>
__device__ __forceinline__ IvT<U> forward_ext(const FmiDevT<U> &f, IvT<U> in, int q)   // q = read base 0..3
{
    IvT<U> sw = {in.l, in.k, in.s};
    IvT<U> o = backward_ext(f, sw, 3 - q);
    return IvT<U>{o.l, o.k, o.s};
}

template <class U>
__device__ __forceinline__ IvT<U> set_intv(const FmiDevT<U> &f, int c)
{
    const U k = f.count[c], k1 = f.count[c + 1], l = f.count[3 - c];
    return IvT<U>{k, l, k1 - k};
}

// k-mer table entries: x, y, z = the low 32 bits of k, l, s; w = their bits 32..39 (wide index)
__device__ __forceinline__ uint64_t ktab_off(int len) { return ((1ull << (2 * len)) - 4) / 3; }
template <class U>
__device__ __forceinline__ uint4 ktab_pack(IvT<U> v)
{
    if constexpr (sizeof(U) == 8)
        return uint4{(uint32_t)v.k, (uint32_t)v.l, (uint32_t)v.s,
                     (uint32_t)((v.k >> 32) & 0xff) | (uint32_t)((v.l >> 32) & 0xff) << 8 |
                         (uint32_t)((v.s >> 32) & 0xff) << 16};
    else
        return uint4{v.k, v.l, v.s, 0u};
}
// the interval of the len-base string with base-4 code `code` (1 <= len <= f.kt)
template <class U>
__device__ __forceinline__ IvT<U> ktab_get(const FmiDevT<U> &f, int len, uint64_t code)
{
    const uint4 e = f.ktab[ktab_off(len) + code];
    if constexpr (sizeof(U) == 8)
        return IvT<U>{(uint64_t)e.x | (uint64_t)(e.w & 0xff) << 32, (uint64_t)e.y | (uint64_t)((e.w >> 8) & 0xff) << 32,
                      (uint64_t)e.z | (uint64_t)((e.w >> 16) & 0xff) << 32};
    else
        return IvT<U>{e.x, e.y, e.z};
}

// 4 bytes at p (any alignment) from aligned dword loads; p .. p + 7 must be readable
__device__ __forceinline__ uint32_t load4u(const uint8_t *p)
{
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
    return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3));
}

// the number of leading j < lim with q[j] == T[tp + j]: the text's 0xFF padding ends a run at
// the text end and a read N (4) never equals a text base
__device__ __forceinline__ int match_run(const uint8_t *__restrict__ T, uint64_t tp, const uint8_t *__restrict__ q,
                                         int lim)
{
    int j = 0;
    while (lim - j >= 8) {
        const uint32_t x = load4u(T + tp + j) ^ load4u(q + j);
        if (x) return j + (__builtin_ctz(x) >> 3);
        j += 4;
    }
    while (j < lim && q[j] == T[tp + j]) ++j;
    return j;
}

// the (k, l) of q[b, e) occurring (once) at text position p: rows of that suffix and of the
// reverse complement's occurrence at n - p - (e - b) (T = ref + revcomp(ref))
template <class U>
__device__ __forceinline__ IvT<U> text_intv(const FmiDevT<U> &f, U p, int len)
{
    return IvT<U>{f.isa[p], f.isa[f.n - p - (U)len], (U)1};
}

// ---------------------------------------------------------------- device: per-read passes

#ifndef BSW_SMEM_KPF
#define BSW_SMEM_KPF 1           // 0: the forward walks issue each table load when they need it
#endif

// The first 16 bases of q[x, len) in registers, and a two-deep pipeline of k-mer table loads over
// its N-free prefix: a forward walk's first steps (one per base, each waiting on its own load)
// then wait on a load issued two steps earlier -- the table loads depend on the read alone.  The
// read's bases come from registers too, since waiting on a byte load of the read would also wait
// for every older load (the memory counter is in order).
template <class U>
struct KPre {
    uint32_t pw;                 // q[x + t] & 3 in bits 31 - 2t .. 30 - 2t
    uint32_t nm;                 // bit t: q[x + t] is N, or x + t >= len
    int P;                       // lengths 1 .. P are table-served: N-free, <= kt
    int m;                       // the length the next take() returns
    bool so;                     // lengths < P load the count alone (FmiDevT::stab)
    bool part;                   // the last take() returned a count alone (k, l unset)
    uint4 e0, e1;                // entries of lengths m, m + 1
    __device__ __forceinline__ int base(int t) const { return (nm >> t & 1) ? 4 : (int)(pw >> (30 - 2 * t) & 3); }
    __device__ __forceinline__ uint4 load(const FmiDevT<U> &f, int len) const
    {
        if (len < P && so) return uint4{0, 0, f.stab[ktab_off(len) + (pw >> (32 - 2 * len))], 0};
        return len <= P ? f.ktab[ktab_off(len) + (pw >> (32 - 2 * len))] : uint4{0, 0, 0, 0};
    }
    // the full interval of q[x, x + len) (len <= P), for a walk that needs k of a count-only entry
    __device__ __forceinline__ IvT<U> full(const FmiDevT<U> &f, int len) const
    {
        return ktab_get(f, len, (uint64_t)(pw >> (32 - 2 * len)));
    }
    // sonly: the caller needs k, l of a table-served walk entry only at length P (its last, which
    // forward_ext continues from and which the sweeps store) or through full()
    __device__ __forceinline__ void init(const FmiDevT<U> &f, const uint8_t *q, int x, int len, bool sonly = false)
    {
        const int nb = min(16, len - x);                         // >= 1
        const uintptr_t a = (uintptr_t)(q + x);
        const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3);
        const int nd = (int)(sh + nb + 3) >> 2;                  // aligned dwords holding a read byte
        uint32_t d[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) d[k] = k < nd ? w[k] : 0xFFFFFFFFu;   // never past a read byte's page
        pw = 0;
        nm = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t r = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);   // q[x + 4j, + 4)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int t = 4 * j + b;
                const uint32_t c = r >> (8 * b) & 0xff;
                nm |= (uint32_t)(t >= nb || c > 3) << t;
                pw |= (c & 3) << (30 - 2 * t);
            }
        }
        P = min(f.kt, (int)__builtin_ctz(nm | 0x10000u));
        so = sonly && f.stab != nullptr;
        part = false;
        m = 2;
        e0 = load(f, 2);
        e1 = load(f, 3);
    }
    // the interval of q[x, x + m) (m <= P), then m + 1
    __device__ __forceinline__ IvT<U> take(const FmiDevT<U> &f)
    {
        const uint4 e = e0;
        part = m < P && so;
        e0 = e1;
        e1 = load(f, m + 2);
        ++m;
        if constexpr (sizeof(U) == 8)
            return IvT<U>{(uint64_t)e.x | (uint64_t)(e.w & 0xff) << 32, (uint64_t)e.y | (uint64_t)((e.w >> 8) & 0xff) << 32,
                          (uint64_t)e.z | (uint64_t)((e.w >> 16) & 0xff) << 32};
        else
            return IvT<U>{e.x, e.y, e.z};
    }
};

template <class U>
struct alignas(16) EntT {            // one interval-vector entry: (k, l, s) and the match end
    U k, l, s, e;
};

// Interval-vector entries in HBM scratch: EntT<U> as is (16 B narrow, 32 B wide), or for the wide
// index the packed 16-B EntP when k, l < 2^40, s < 2^32 and ends < 2^15 (every realistic genome:
// a 3 Gb two-strand text has 6e9 rows and single-base counts ~1.8e9; the host checks and falls
// back to EntT).  The sweeps write and re-read ~20 KB of entries per 150 bp read at 3 Gb (PMC:
// 20 GB of HBM writes per 1M-read launch), so halving the wide entry halves that traffic.
struct alignas(16) EntP {
    uint32_t k, l, s, w;     // w: k bits 32..39, l bits 32..39, e (15 bits + the text flag)
};
template <class U>
__device__ __forceinline__ void ent_put(EntT<U> *p, const EntT<U> &e) { *p = e; }
template <class U>
__device__ __forceinline__ EntT<U> ent_get(const EntT<U> *p) { return *p; }
__device__ __forceinline__ void ent_put(EntP *p, const EntT<uint64_t> &e)
{
    const uint32_t ee = (uint32_t)e.e;
    *reinterpret_cast<uint4 *>(p) = uint4{(uint32_t)e.k, (uint32_t)e.l, (uint32_t)e.s,
                                          (uint32_t)(e.k >> 32 & 0xff) | (uint32_t)(e.l >> 32 & 0xff) << 8 |
                                              (ee & 0x7fffu) << 16 | (ee >> 31) << 31};
}
__device__ __forceinline__ EntT<uint64_t> ent_get(const EntP *p)
{
    const uint4 v = *reinterpret_cast<const uint4 *>(p);
    return EntT<uint64_t>{(uint64_t)v.x | (uint64_t)(v.w & 0xff) << 32, (uint64_t)v.y | (uint64_t)(v.w >> 8 & 0xff) << 32,
                          (uint64_t)v.z, (uint64_t)((v.w >> 16 & 0x7fffu) | (v.w >> 31) << 31)};
}

// The interval vectors' first kSmemLds entries live in LDS, [vector][slot][lane] as 16-B words (one
// ds_read/write_b128 per entry, conflict-free), the rest in the HBM scratch: by the PMC of a 3 Gb
// launch the sweeps' write-then-re-read of the vectors was most of the walk's ~55 KB fetched per read
// (DESIGN.md §8).  8 KB of LDS per one-wave workgroup at 4 slots (16-B entries only; 0 = off).
#ifndef BSW_SMEM_LDS
#define BSW_SMEM_LDS 4
#endif
#ifndef BSW_SMEM_VIRT
#define BSW_SMEM_VIRT 1          // 0: every interval-vector entry stored (smem1's virtual entries off)
#endif
constexpr int kSmemLds = BSW_SMEM_LDS;
// the narrow (32-bit) index's walk: no LDS slots and 5 waves per SIMD (16 Mb, with virtual entries:
// 74.4 vs 71.1 M reads/s without the slots, 73.2 at 5 waves, profiles/r05/smem_virtual_entries_ab.txt)
#ifndef BSW_SMEM_LDS_NARROW
#define BSW_SMEM_LDS_NARROW 0
#endif
#ifndef BSW_SMEM_WAVES_NARROW
#define BSW_SMEM_WAVES_NARROW 5
#endif
// the wide (64-bit) walk at 5 waves too since its stored extensions go one at a time (96 VGPRs, 4
// spilled; LDS 5 x 4 x 8 KB = the CU's 160 KB): C4 207.4 / 207.9 -> 204.2 / 204.9 ms per step
#ifndef BSW_SMEM_WAVES_WIDE
#define BSW_SMEM_WAVES_WIDE 5
#endif
template <class U, class S>
constexpr int lds_slots() { return sizeof(S) != 16 ? 0 : sizeof(U) == 8 ? kSmemLds : BSW_SMEM_LDS_NARROW; }

template <class U, class S = EntT<U>>
struct Lane {
    const uint8_t *q;
    int len;
    uint4 *lds;              // this lane's LDS slots: [v][j] at lds[(v * K + j) * 64], K = lds_slots (or nullptr)
    S *sa, *sb;              // scratch vectors, element j at [j * stride]
    size_t stride;
    int scap;                // scratch entries per vector
    bsw_bwtintv_t *out;      // this read's output slots
    int cap;
    int nout;                // intervals produced (may exceed cap)
    int overflow;            // scratch overflow (cannot happen for scap >= len + 1)
};

template <class U, class S>
__device__ __forceinline__ void push_out(Lane<U, S> &L, IvT<U> v, uint32_t start, uint32_t end)
{
    if (L.nout < L.cap) {
        bsw_bwtintv_t o;
        o.x[0] = v.k; o.x[1] = v.l; o.x[2] = v.s;
        o.info = ((uint64_t)start << 32) | end;
        L.out[L.nout] = o;
    }
    ++L.nout;
}

// vector v (0: sa, 1: sb), entry j
template <class U, class S>
__device__ __forceinline__ void vput(Lane<U, S> &L, int v, int j, const EntT<U> &e)
{
    constexpr int K = lds_slots<U, S>();
    if constexpr (K > 0) {
        if (j < K) {
            S t;
            ent_put(&t, e);
            L.lds[(v * K + j) * 64] = *reinterpret_cast<const uint4 *>(&t);
            return;
        }
    }
    ent_put((v ? L.sb : L.sa) + (size_t)j * L.stride, e);
}
template <class U, class S>
__device__ __forceinline__ EntT<U> vget(const Lane<U, S> &L, int v, int j)
{
    constexpr int K = lds_slots<U, S>();
    if constexpr (K > 0) {
        if (j < K) {
            S t;
            *reinterpret_cast<uint4 *>(&t) = L.lds[(v * K + j) * 64];
            return ent_get(&t);
        }
    }
    return ent_get((v ? L.sb : L.sa) + (size_t)j * L.stride);
}

// bwt_smem1a with max_intv = 0 (bwt_smem1): SMEMs overlapping x with occurrence >= min_intv;
// those of length >= keep_len go to the output.  Returns the next x.
//
// prune (the re-seeding pass, whose return value is unused): every interval the backward sweep
// could output is a substring q[b, e) with >= min_intv occurrences that contains x, so its suffix
// q[x, e) and its prefix q[b, x] have >= min_intv occurrences too (occurrences only shrink as a
// string grows): e <= e_max, the forward reach the forward phase has just found, and b >= b_min,
// the backward reach of the single base q[x].  When e_max - b_min < keep_len nothing can be
// output and the sweep (~8x the forward phase's block loads on a genome: every entry extended
// until its count drops) is skipped -- outputs identical by construction (re-seeding of unique
// SMEMs on a large genome almost never finds a >= 19-base repeat).
template <class U, class S>
__device__ int smem1(const FmiDevT<U> &f, Lane<U, S> &L, int x, U min_intv, int keep_len, bool prune = false)
{
    const uint8_t *q = L.q;
    const int len = L.len;
    const int qx = q[x];
    if (qx > 3) return x + 1;
    if (min_intv < 1) min_intv = 1;
    int curr = 0, prev = 1;                               // vector ids (vput / vget)
    IvT<U> ik = set_intv(f, qx);
    bool ik_part = false;                                 // ik holds its count alone (KPre::part)
    U ikend = (U)(x + 1);
    int nc = 0, i;
    const bool text = f.text && min_intv <= 1;
    // Virtual entries: an entry whose string the next sweep step extends from the k-mer table
    // (extension length b = pe - i <= kt at the reading step i) needs none of its (k, l, s) -- the
    // table entry of q[i, pe) comes from the read's 2-bit window -- and is never output (its length
    // b - 1 < keep_len), so it is kept as bit b of a per-vector mask instead of a 16-B entry.  The
    // vectors are ordered by descending pe in sweep order, so the stored entries are exactly the
    // leading ones (b > vmax) and the mask holds the tail.  0 = off (no table, or keep_len < kt).
    const int vmax = (BSW_SMEM_VIRT && keep_len >= f.kt) ? f.kt : 0;
    uint32_t vmask = 0;                                    // forward entries, bit b: pe = x - 1 + b
    int nf = 0;                                           // forward entries stored
    auto fpush = [&](U e) {
        const int b = (int)((uint32_t)e & ~kTextFlag) - (x - 1);
        if (b <= vmax) {
            vmask |= 1u << b;
        } else {
            if (nf < L.scap) vput(L, curr, nf, EntT<U>{ik.k, ik.l, ik.s, e});
            else L.overflow = 1;
            ++nf;
        }
        ++nc;
    };
#if BSW_SMEM_KPF
    // with virtual entries every forward push shorter than kt is virtual (s alone matters), so the
    // table loads below P fetch counts only; k, l come from the full table at P or on demand
    KPre<U> pre;
    pre.init(f, q, x, len, vmax > 0);
    uint64_t win = (uint64_t)pre.pw << 32;              // q[x, x + 16), q[x] in bits 63:62 (the sweep)
#else
    // q[x, i) as a base-4 code (table lookups while i + 1 - x <= kt) and as a 2-bit window with
    // q[x] in bits 63:62 (the backward sweep's table lookups)
    uint64_t code = (uint64_t)qx, win = (uint64_t)qx << 62;
#endif
    for (i = x + 1; i < len; ++i) {                      // forward search
        if (text && ik.s == 1) {
            // one occurrence left: every further step keeps s = 1 while the read matches the
            // text after it, and the first step that does not (mismatch, read N, text end) pushes
            // ik and stops -- so compare read and text directly, then push ik as a text-mode
            // entry (its k, l are only needed if it is output)
#if BSW_SMEM_KPF
            if (ik_part) ik = pre.full(f, i - x);           // a count-only table entry: its k
#endif
            const U p = f.sa[ik.k];
            const int e = i + match_run(f.text, (uint64_t)p + (uint64_t)(i - x), q + i, len - i);
            ik.k = p;
            ikend = (U)((uint32_t)e | kTextFlag);
            if (e < len) fpush(ikend);
            i = e;
            break;
        }
#if BSW_SMEM_KPF
        const int qi = i - x < 16 ? pre.base(i - x) : q[i];
        if (qi < 4) {
            const bool tk = i + 1 - x <= pre.P;
            const IvT<U> ok = tk ? pre.take(f) : forward_ext(f, ik, qi);
            const bool ok_part = tk && pre.part;
#else
        const int qi = q[i];
        if (qi < 4) {
            code = code << 2 | (uint64_t)qi;
            if (i - x < 32) win |= (uint64_t)qi << (62 - 2 * (i - x));
            const IvT<U> ok = i + 1 - x <= f.kt ? ktab_get(f, i + 1 - x, code) : forward_ext(f, ik, qi);
            const bool ok_part = false;
#endif
            if (ok.s != ik.s) {
                fpush(ikend);
                if (ok.s < min_intv) break;
            }
            ik = ok; ik_part = ok_part; ikend = (U)(i + 1);
        } else {
            fpush(ikend);
            break;
        }
    }
    if (i == len) fpush(ikend);
    nf = min(nf, L.scap);
    // upstream reverses curr (longest matches first); here prev is read back to front once.  The
    // longest match is the last stored entry, or the mask's highest bit when none is stored
    const int ret = nf > 0 ? (int)((uint32_t)vget(L, curr, nf - 1).e & ~kTextFlag)
                           : x - 1 + (31 - __builtin_clz(vmask));
    if (prune && ret - x < keep_len) {
        // b_min: extend q[x] to the left while it keeps >= min_intv occurrences; stop as soon as
        // the bound reaches keep_len (then the sweep must run)
        IvT<U> bk = set_intv(f, qx);
        int b = x;
        uint64_t bcode = (uint64_t)qx;                   // q[b, x] as a base-4 code
        while (b > 0 && ret - b < keep_len) {
            const int c = q[b - 1];
            if (c > 3) break;
            const int m = x + 2 - b;                     // length of q[b - 1, x]
            if (m <= f.kt) bcode |= (uint64_t)c << (2 * (m - 1));   // (kt <= 15: the shift stays < 64)
            // (only s matters below kt: bk is extended by blocks only once m > kt)
            const IvT<U> ok = (m < f.kt && f.stab) ? IvT<U>{0, 0, (U)f.stab[ktab_off(m) + bcode]}
                              : m <= f.kt ? ktab_get(f, m, bcode) : backward_ext(f, bk, c);
            if (ok.s < min_intv) break;
            bk = ok;
            --b;
        }
        if (ret - b < keep_len) return ret;
    }
    { const int t = curr; curr = prev; prev = t; }
    int np = nf;                                          // prev: stored entries, then the mask
    uint32_t pmask = vmask;                               // bit b: pe = i + b at the reading step i
    bool rev = true;
    int nmem = 0;
    uint32_t last_start = 0;
    for (i = x - 1; i >= -1; --i) {                      // backward search
        const int c = i < 0 ? -1 : (q[i] < 4 ? q[i] : -1);
        win = win >> 2 | (uint64_t)(c & 3) << 62;      // q[i, i + 32)
        nc = 0;
        int ncf = 0;                                      // curr entries stored
        uint32_t cmask = 0;                               // curr entries virtual (bit pe - i + 1)
        U last_cs = 0;
        // the entries' extensions are independent loads: compute kBackUnroll of them before
        // their (sequential, order-dependent) bookkeeping, so a lane has that many block loads in
        // flight instead of one
        auto ext_of = [&](const EntT<U> &pv) -> IvT<U> {
            IvT<U> ok = {0, 0, 0};
            if (c >= 0) {
                const int m = (int)((uint32_t)pv.e & ~kTextFlag) - i;   // length of q[i, pe)
                if ((uint32_t)pv.e & kTextFlag) {           // one occurrence: the base before it
                    if (pv.k > 0 && f.text[pv.k - 1] == (uint8_t)c) ok = IvT<U>{pv.k - 1, 0, 1};
                } else if (m <= f.kt) {                     // a short string: its table entry
                    ok = ktab_get(f, m, win >> (64 - 2 * m));
                } else {
                    ok = backward_ext(f, IvT<U>{pv.k, pv.l, pv.s}, c);
                }
            }
            return ok;
        };
        // bwt_smem1a's per-entry bookkeeping, in vector order (stored entries, then virtual ones)
        auto book = [&](const EntT<U> &pv, const IvT<U> &ok) {
            const bool tm = ((uint32_t)pv.e & kTextFlag) != 0;   // text mode: pv.k = text position
            const uint32_t pe = (uint32_t)pv.e & ~kTextFlag;
            if (c < 0 || ok.s < min_intv) {
                if (nc == 0) {
                    if (nmem == 0 || (uint32_t)(i + 1) < last_start) {
                        last_start = (uint32_t)(i + 1);
                        ++nmem;
                        if ((int)(pe - last_start) >= keep_len)   // (never a virtual entry)
                            push_out(L, tm ? text_intv(f, pv.k, (int)(pe - last_start)) : IvT<U>{pv.k, pv.l, pv.s},
                                     last_start, pe);
                    }
                }
            } else if (nc == 0 || ok.s != last_cs) {
                const int b = (int)pe - i + 1;                 // its extension length at step i - 1
                if (b <= vmax) {
                    cmask |= 1u << b;
                } else {
                    // an interval down to one occurrence continues in text mode (one SA load now,
                    // then cached text reads instead of occurrence blocks)
                    const bool to_text = f.text && ok.s == 1;
                    const U k2 = tm ? ok.k : (to_text ? f.sa[ok.k] : ok.k);
                    if (ncf < L.scap)
                        vput(L, curr, ncf, EntT<U>{k2, ok.l, ok.s, (U)(pe | ((tm || to_text) ? kTextFlag : 0u))});
                    else L.overflow = 1;
                    ++ncf;
                }
                ++nc;
                last_cs = ok.s;
            }
        };
        for (int j0 = 0; j0 < np; j0 += kBackUnroll) {
          EntT<U> pvs[kBackUnroll];
          IvT<U> oks[kBackUnroll];
#pragma unroll
          for (int u = 0; u < kBackUnroll; ++u) {
              const int j = min(j0 + u, np - 1);
              pvs[u] = vget(L, prev, rev ? np - 1 - j : j);
          }
#pragma unroll
          for (int u = 0; u < kBackUnroll; ++u) oks[u] = ext_of(pvs[u]);
#pragma unroll
          for (int u = 0; u < kBackUnroll; ++u) {
            if (j0 + u >= np) break;
            book(pvs[u], oks[u]);
          }
        }
        for (uint32_t mm = pmask; mm != 0;) {             // the virtual entries, longest first
          int bs[kVirtUnroll];
          IvT<U> oks[kVirtUnroll];
#pragma unroll
          for (int u = 0; u < kVirtUnroll; ++u) {
              bs[u] = mm ? 31 - __builtin_clz(mm) : 0;
              mm &= ~(1u << bs[u]);
          }
#pragma unroll
          for (int u = 0; u < kVirtUnroll; ++u)
              // below vmax the extension stays virtual (only its s matters): the counts-only table
              oks[u] = (c >= 0 && bs[u] > 0)
                           ? ((bs[u] < vmax && f.stab)
                                  ? IvT<U>{0, 0, (U)f.stab[ktab_off(bs[u]) + (win >> (64 - 2 * bs[u]))]}
                                  : ktab_get(f, bs[u], win >> (64 - 2 * bs[u])))
                           : IvT<U>{0, 0, 0};
#pragma unroll
          for (int u = 0; u < kVirtUnroll; ++u) {
            if (bs[u] == 0) break;
            book(EntT<U>{0, 0, 0, (U)(i + bs[u])}, oks[u]);
          }
        }
        if (nc == 0) break;
        np = min(ncf, L.scap);
        pmask = cmask;
        rev = false;
        { const int t = curr; curr = prev; prev = t; }
    }
    return ret;
}

// bwt_seed_strategy1
template <class U, class S>
__device__ int seed_strategy1(const FmiDevT<U> &f, Lane<U, S> &L, int x, int min_len, U max_intv)
{
    const uint8_t *q = L.q;
    const int qx = q[x];
    if (qx > 3) return x + 1;
    IvT<U> ik = set_intv(f, qx);
    bool ik_part = false;                                 // ik holds its count alone (KPre::part)
#if BSW_SMEM_KPF
    // outputs are >= min_len > kt bases long: below P the walk needs counts only
    KPre<U> pre;
    pre.init(f, q, x, L.len, min_len > f.kt);
#else
    uint64_t code = (uint64_t)qx;                        // q[x, i) as a base-4 code
#endif
    for (int i = x + 1; i < L.len; ++i) {
        if (f.text && ik.s == 1 && max_intv > 1) {
            // one occurrence: the walk returns at i* = max(i, x + min_len) (every s is 0 or 1 <
            // max_intv) unless a read N comes first; it pushes the interval if the read still
            // matches the text through i*
            const int is = max(i, x + min_len);
            int t = i;
            const int lim = min(is + 1, L.len);
            while (t < lim && q[t] < 4) ++t;                 // first N in [i, is]
            if (t < lim) return t + 1;
            if (is >= L.len) return L.len;
#if BSW_SMEM_KPF
            if (ik_part) ik = pre.full(f, i - x);           // a count-only table entry: its k
#endif
            const U p = f.sa[ik.k];
            if (match_run(f.text, (uint64_t)p + (uint64_t)(i - x), q + i, is + 1 - i) == is + 1 - i)
                push_out(L, text_intv(f, p, is + 1 - x), (uint32_t)x, (uint32_t)(is + 1));
            return is + 1;
        }
#if BSW_SMEM_KPF
        const int qi = i - x < 16 ? pre.base(i - x) : q[i];
        if (qi < 4) {
            const bool tk = i + 1 - x <= pre.P;
            const IvT<U> ok = tk ? pre.take(f) : forward_ext(f, ik, qi);
            const bool ok_part = tk && pre.part;
#else
        const int qi = q[i];
        if (qi < 4) {
            code = code << 2 | (uint64_t)qi;
            const IvT<U> ok = i + 1 - x <= f.kt ? ktab_get(f, i + 1 - x, code) : forward_ext(f, ik, qi);
            const bool ok_part = false;
#endif
            if (ok.s < max_intv && i - x >= min_len) {
                if (ok.s > 0) push_out(L, ok, (uint32_t)x, (uint32_t)(i + 1));
                return i + 1;
            }
            ik = ok;
            ik_part = ok_part;
        } else {
            return i + 1;
        }
    }
    return L.len;
}

__device__ __forceinline__ bool iv_less(const bsw_bwtintv_t &a, const bsw_bwtintv_t &b)
{
    if (a.info != b.info) return a.info < b.info;
    if (a.x[0] != b.x[0]) return a.x[0] < b.x[0];
    if (a.x[2] != b.x[2]) return a.x[2] < b.x[2];
    return a.x[1] < b.x[1];
}

// one read's mem_collect_intv (lane t of a launch over reads n0 .. n0 + n - 1): returns error
// bits (1: more than cap intervals, 2: bad length / scratch overflow).  Plain loops, as upstream
// writes them: a per-lane state machine doing one extension per iteration (so that a wave's time
// is its busiest lane's work instead of the sum of per-phase maxima) measured 1.4x SLOWER (31.9
// vs 22.1 ms on 1M reads x 16 Mb) -- the bookkeeping transitions cost whole iterations.
template <class U, class S>
__device__ int smem_read(const FmiDevT<U> &f, const MemOpt &opt, const uint8_t *__restrict__ reads,
                         const int64_t *__restrict__ read_off, const int32_t *__restrict__ read_len, int32_t n0,
                         int32_t n, int t, S *__restrict__ scratch, int32_t scap,
                         bsw_bwtintv_t *__restrict__ mems, int32_t cap, int32_t *__restrict__ n_mems,
                         uint4 *lds)
{
    const int r = n0 + t;                                    // read index
    Lane<U, S> L;
    L.lds = lds;
    L.q = reads + read_off[r];
    L.len = read_len[r];
    // [slot][read]: a wave's lanes at the same slot touch one contiguous run (a [read][slot] layout,
    // each read's vectors contiguous, measured 13% slower at 3 Gb: profiles/r04/hostpath_ab_r4m.txt)
    L.stride = (size_t)n;
    L.sa = scratch + t;
    L.sb = scratch + (size_t)scap * n + t;
    L.scap = scap;
    L.out = mems + (size_t)r * cap;
    L.cap = cap;
    L.nout = 0;
    L.overflow = 0;
    if (L.len < 0 || L.len > scap - 1) {
        n_mems[r] = 0;
        return 2;
    }
    // pass 1: SMEMs
    int x = 0;
    while (x < L.len) {
        if (L.q[x] < 4) x = smem1(f, L, x, (U)1, opt.min_seed_len);
        else ++x;
    }
    // pass 2: re-seeding inside long SMEMs of few occurrences
    const int old_n = min(L.nout, cap);
    for (int k = 0; k < old_n; ++k) {
        const bsw_bwtintv_t p = L.out[k];
        const int start = (int)(p.info >> 32), end = (int)(uint32_t)p.info;
        if (end - start < opt.split_len || p.x[2] > (uint64_t)opt.split_width) continue;
        smem1(f, L, (start + end) >> 1, (U)(p.x[2] + 1), opt.min_seed_len, true);
    }
    // pass 3: LAST-like seeds
    if (opt.max_mem_intv > 0) {
        x = 0;
        while (x < L.len) {
            if (L.q[x] < 4) x = seed_strategy1(f, L, x, opt.min_seed_len, (U)opt.max_mem_intv);
            else ++x;
        }
    }
    // sort by (info, k, s, l)
    const int m = min(L.nout, cap);
    for (int a = 1; a < m; ++a) {
        const bsw_bwtintv_t v = L.out[a];
        int b = a - 1;
        while (b >= 0 && iv_less(v, L.out[b])) {
            L.out[b + 1] = L.out[b];
            --b;
        }
        L.out[b + 1] = v;
    }
    n_mems[r] = L.nout;
    return (L.nout > cap ? 1 : 0) | (L.overflow ? 2 : 0);
}

#ifndef BSW_SMEM_BLOCK
#define BSW_SMEM_BLOCK 64
#endif
constexpr int kSmemBlock = BSW_SMEM_BLOCK;          // threads per workgroup of the SMEM kernel

template <class U, class S>
#ifndef BSW_SMEM_WAVES           // experiment builds: a minimum of waves per SIMD for the walk
#define BSW_SMEM_WAVES 0         // (0 = the compiler's choice: 4 wide / 6 narrow)
#endif
#if BSW_SMEM_WAVES > 0
#define BSW_SMEM_LB __launch_bounds__(kSmemBlock, BSW_SMEM_WAVES)
#else
#define BSW_SMEM_LB __launch_bounds__(kSmemBlock, sizeof(U) == 4 ? BSW_SMEM_WAVES_NARROW : BSW_SMEM_WAVES_WIDE)
#endif
__global__ BSW_SMEM_LB void smem_kernel(const FmiDevT<U> f, const MemOpt opt,
                                                  const uint8_t *__restrict__ reads,
                                                  const int64_t *__restrict__ read_off,
                                                  const int32_t *__restrict__ read_len, int32_t n0, int32_t n,
                                                  S *__restrict__ scratch, int32_t scap,
                                                  bsw_bwtintv_t *__restrict__ mems, int32_t cap,
                                                  int32_t *__restrict__ n_mems, int32_t *__restrict__ err)
{
    constexpr int K = lds_slots<U, S>();
    static_assert(kSmemBlock == 64 || K == 0, "LDS vector slots assume one wave per workgroup");
    __shared__ uint4 s_vec[K > 0 ? 2 * K * 64 : 1];
    const int t = blockIdx.x * blockDim.x + threadIdx.x;    // lane within this chunk
    if (t >= n) return;
    const int e = smem_read(f, opt, reads, read_off, read_len, n0, n, t, scratch, scap, mems, cap, n_mems,
                            K > 0 ? s_vec + (threadIdx.x & 63) : nullptr);
    if (e) atomicOr(err, e);
}

// one level of the k-mer interval table: level 1 from the counts, level j > 1 by extending every
// level-(j - 1) entry backward by its first base (a string's interval is unique, so this equals
// what the walks compute step by step); grid-stride (an AQL grid is 32-bit)
template <class U>
__global__ void ktab_kernel(const FmiDevT<U> f, int j, uint4 *__restrict__ tab)
{
    const uint64_t cnt = 1ull << (2 * j), o = ktab_off(j);
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += (uint64_t)gridDim.x * blockDim.x) {
        IvT<U> v;
        if (j == 1) {
            v = set_intv(f, (int)c);
        } else {
            const uint64_t rest = c & ((1ull << (2 * (j - 1))) - 1);
            const uint4 e = tab[ktab_off(j - 1) + rest];
            IvT<U> p;
            if constexpr (sizeof(U) == 8)
                p = IvT<U>{(uint64_t)e.x | (uint64_t)(e.w & 0xff) << 32, (uint64_t)e.y | (uint64_t)((e.w >> 8) & 0xff) << 32,
                           (uint64_t)e.z | (uint64_t)((e.w >> 16) & 0xff) << 32};
            else
                p = IvT<U>{e.x, e.y, e.z};
            v = backward_ext(f, p, (int)(c >> (2 * (j - 1))));
        }
        tab[o + c] = ktab_pack(v);
    }
}

// the k-mer table's counts alone (s < 2^32: the host checks the single-base counts), grid-stride
__global__ void stab_kernel(const uint4 *__restrict__ tab, uint64_t ents, uint32_t *__restrict__ stab)
{
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < ents; c += (uint64_t)gridDim.x * blockDim.x)
        stab[c] = tab[c].z;
}

template <class S>
__global__ void sa_kernel(const S *__restrict__ sa, uint64_t nrows, const uint64_t *__restrict__ k, int64_t n,
                          int64_t *__restrict__ pos)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t r = k[i];
    pos[i] = r < nrows ? (int64_t)sa[r] : -1;
}

// ---------------------------------------------------------------- host: suffix array

// LSD radix sort of (key, idx) by key, 16-bit digits over the bits that can be set
void radix_sort64(std::vector<uint64_t> &key, std::vector<uint32_t> &idx, int bits)
{
    const size_t n = key.size();
    std::vector<uint64_t> k2(n);
    std::vector<uint32_t> i2(n);
    std::vector<size_t> cnt(1 << 16);
    for (int sh = 0; sh < bits; sh += 16) {
        std::fill(cnt.begin(), cnt.end(), 0);
        for (size_t i = 0; i < n; ++i) cnt[(key[i] >> sh) & 0xffff]++;
        size_t acc = 0;
        for (auto &c : cnt) { const size_t t = c; c = acc; acc += t; }
        for (size_t i = 0; i < n; ++i) {
            const size_t d = cnt[(key[i] >> sh) & 0xffff]++;
            k2[d] = key[i];
            i2[d] = idx[i];
        }
        key.swap(k2);
        idx.swap(i2);
    }
}

// suffix array of T$ (t = codes 0..3, length n); sa has n + 1 entries
void build_sa(const uint8_t *t, uint32_t n, std::vector<uint32_t> &sa)
{
    const uint32_t N = n + 1;
    constexpr int H0 = 27;                                   // 5^27 < 2^63
    std::vector<uint64_t> key(N);
    {
        uint64_t p26 = 1;
        for (int d = 0; d < H0 - 1; ++d) p26 *= 5;
        uint64_t k = 0;
        for (int64_t i = (int64_t)N - 1; i >= 0; --i) {      // key[i] = c(i) 5^26 + key[i + 1] / 5
            const uint64_t c = (uint64_t)i < n ? (uint64_t)t[i] + 1 : 0;
            k = c * p26 + k / 5;
            key[i] = k;
        }
    }
    sa.resize(N);
    for (uint32_t i = 0; i < N; ++i) sa[i] = i;
    radix_sort64(key, sa, 64);
    std::vector<uint32_t> rank(N);
    std::vector<std::pair<uint32_t, uint32_t>> groups;       // [start, end) tie groups
    for (uint32_t j = 0; j < N;) {
        uint32_t e = j + 1;
        while (e < N && key[e] == key[j]) ++e;
        for (uint32_t u = j; u < e; ++u) rank[sa[u]] = j;
        if (e - j > 1) groups.emplace_back(j, e);
        j = e;
    }
    std::vector<uint64_t>().swap(key);
    std::vector<std::pair<uint32_t, uint32_t>> tmp, next;
    for (uint64_t h = H0; !groups.empty(); h *= 2) {
        next.clear();
        for (const auto &g : groups) {
            tmp.clear();
            for (uint32_t u = g.first; u < g.second; ++u) {
                const uint64_t p = (uint64_t)sa[u] + h;     // < N inside a tie group ('$' is unique)
                tmp.emplace_back(p < N ? rank[p] : 0u, sa[u]);
            }
            std::sort(tmp.begin(), tmp.end());
            for (uint32_t u = 0; u < tmp.size(); ++u) sa[g.first + u] = tmp[u].second;
            for (uint32_t u = 0; u < tmp.size();) {
                uint32_t e = u + 1;
                while (e < tmp.size() && tmp[e].first == tmp[u].first) ++e;
                for (uint32_t v = u; v < e; ++v) rank[tmp[v].second] = g.first + u;
                if (e - u > 1) next.emplace_back(g.first + u, g.first + e);
                u = e;
            }
        }
        groups.swap(next);
    }
}

}  // namespace

struct bsw_fmi {
    int device = 0;
    int64_t n = 0;                            // |T|
    bool wide = false;                        // 64-bit rows / counts / suffix array
    bool gpu_built = false;
    bool plain_ent = false;                   // BSW_FMI_PLAIN_ENT: 32-B interval-vector entries always
    FmiDevT<uint32_t> dv32{};
    FmiDevT<uint64_t> dv64{};
    void *d_blk = nullptr;                    // FmiBlock (narrow) or FmiBlockW (wide)
    void *d_sa = nullptr;                     // uint32_t (narrow) or uint64_t (wide)
    uint8_t *d_bwt = nullptr;                 // GPU-built index: BWT codes (copy_bwt)
    uint8_t *d_text = nullptr;                // text mode: T + 64 bytes of 0xFF padding
    void *d_isa = nullptr;                    // text mode: SA^-1 (uint32_t or uint64_t)
    uint4 *d_ktab = nullptr;                  // k-mer interval table (levels 1 .. kt)
    uint32_t *d_stab = nullptr;               // its counts s alone (FmiDevT::stab)
    int kt = 0;
    std::vector<uint32_t> sa;                 // host-built index: host copies (tests, bwt_sa)
    std::vector<FmiBlock> h_blk;              // host-only index (device < 0): the occurrence blocks
    std::vector<uint8_t> bwt;
    int64_t count[5] = {0, 0, 0, 0, 0};
    int64_t sentinel = 0;
    int64_t dev_bytes = 0;
    int64_t tie_groups = 0;
    float build_s = 0, kernel_ms = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    void *d_scratch = nullptr;
    size_t scratch_bytes = 0;
    int32_t *d_err = nullptr;
    void *h_stage = nullptr;                  // host-buffer calls: device copies
    std::mutex mu;                            // one seeding call at a time per index
};

int bsw::fmi_view(bsw_fmi_t *f, FmiView *out)
{
    if (!f) return BSW_E_INVAL;
    if (f->device < 0) return BSW_E_NODEV;
    *out = FmiView{f->device, f->d_sa, f->wide, f->n, f->n / 2, f->stream, &f->mu};
    return BSW_OK;
}

namespace {

int hip_rc(hipError_t e) { return e == hipSuccess ? BSW_OK : (e == hipErrorOutOfMemory ? BSW_E_NOMEM : BSW_E_HIP); }

template <class U>
int launch_collect(bsw_fmi_t *f, const FmiDevT<U> &dv, const MemOpt &mo, const uint8_t *d_reads, const int64_t *d_off,
                   const int32_t *d_len, int32_t n, int32_t max_len, bsw_bwtintv_t *d_mems, int32_t cap,
                   int32_t *d_cnt, hipStream_t s)
{
    const int32_t scap = max_len + 1;
    // the wide index's packed 16-B entries when every value fits (EntP); else EntT<U>
    bool packed = false;
    if constexpr (sizeof(U) == 8) {
        uint64_t smax = 0;
        for (int c = 0; c < 4; ++c) smax = std::max<uint64_t>(smax, (uint64_t)(f->count[c + 1] - f->count[c]));
        packed = smax < (1ull << 32) && (uint64_t)f->n + 2 < (1ull << 40) && max_len < 32767 && !f->plain_ent;
    }
    const size_t esz = packed ? sizeof(EntP) : sizeof(EntT<U>);
    // chunk so the two scratch vectors stay within 16 GB (of 288 GB: one launch for up to ~3M
    // 151-bp reads with 16-byte entries)
    const size_t per_read = (size_t)2 * scap * esz;
    const int32_t chunk = (int32_t)std::max<size_t>(64, std::min<size_t>((size_t)n, ((size_t)16 << 30) / per_read));
    const size_t need = per_read * (size_t)std::min(chunk, n);
    if (need > f->scratch_bytes) {
        if (f->d_scratch) (void)hipFree(f->d_scratch);
        f->d_scratch = nullptr;
        f->scratch_bytes = 0;
        if (hipMalloc(&f->d_scratch, need) != hipSuccess) return BSW_E_NOMEM;
        f->scratch_bytes = need;
    }
    if (hipMemsetAsync(f->d_err, 0, sizeof(int32_t), s) != hipSuccess) return BSW_E_HIP;
    (void)hipEventRecord(f->ev0, s);
    for (int32_t n0 = 0; n0 < n; n0 += chunk) {
        const int32_t m = std::min(chunk, n - n0);
        const dim3 grid((unsigned)((m + kSmemBlock - 1) / kSmemBlock));
        if constexpr (sizeof(U) == 8) {
            if (packed)
                hipLaunchKernelGGL((smem_kernel<U, EntP>), grid, dim3(kSmemBlock), 0, s, dv, mo, d_reads, d_off, d_len, n0,
                                   m, (EntP *)f->d_scratch, scap, d_mems, cap, d_cnt, f->d_err);
            else
                hipLaunchKernelGGL((smem_kernel<U, EntT<U>>), grid, dim3(kSmemBlock), 0, s, dv, mo, d_reads, d_off, d_len,
                                   n0, m, (EntT<U> *)f->d_scratch, scap, d_mems, cap, d_cnt, f->d_err);
        } else {
            hipLaunchKernelGGL((smem_kernel<U, EntT<U>>), grid, dim3(kSmemBlock), 0, s, dv, mo, d_reads, d_off, d_len, n0,
                               m, (EntT<U> *)f->d_scratch, scap, d_mems, cap, d_cnt, f->d_err);
        }
        if (hipGetLastError() != hipSuccess) return BSW_E_HIP;
    }
    (void)hipEventRecord(f->ev1, s);
    int32_t herr = 0;
    if (hipMemcpyAsync(&herr, f->d_err, sizeof(int32_t), hipMemcpyDeviceToHost, s) != hipSuccess) return BSW_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return BSW_E_HIP;
    (void)hipEventElapsedTime(&f->kernel_ms, f->ev0, f->ev1);
    return herr ? BSW_E_RANGE : BSW_OK;
}

int run_collect(bsw_fmi_t *f, const bsw_mem_opt_t *opt, const uint8_t *d_reads, const int64_t *d_off,
                const int32_t *d_len, int32_t n, int32_t max_len, bsw_bwtintv_t *d_mems, int32_t cap,
                int32_t *d_cnt, hipStream_t s)
{
    MemOpt mo;
    mo.min_seed_len = opt->min_seed_len;
    mo.split_width = opt->split_width;
    mo.max_mem_intv = opt->max_mem_intv;
    mo.split_len = (int)(opt->min_seed_len * opt->split_factor + .499);
    return f->wide ? launch_collect(f, f->dv64, mo, d_reads, d_off, d_len, n, max_len, d_mems, cap, d_cnt, s)
                   : launch_collect(f, f->dv32, mo, d_reads, d_off, d_len, n, max_len, d_mems, cap, d_cnt, s);
}

// the runtime objects every device index needs
// text mode (BSW_FMI_NO_TEXT off): T = ref + revcomp(ref) with 0xFF padding, and SA^-1
__global__ void k_text_pad(const uint8_t *__restrict__ ref, int64_t len, uint8_t *__restrict__ T)
{
    const int64_t n = 2 * len;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len + 64;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (i < len) {
            const uint8_t c = ref[i];
            T[i] = c;
            T[n - 1 - i] = (uint8_t)(3 - c);
        } else {
            T[n + (i - len)] = 0xFF;
        }
    }
}
template <class S>
__global__ void k_isa(const S *__restrict__ sa, int64_t N, S *__restrict__ isa)
{
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N; r += (int64_t)gridDim.x * blockDim.x)
        isa[sa[r]] = (S)r;
}

int attach_text(bsw_fmi_t *f, const uint8_t *ref, int64_t len)
{
    const int64_t n = f->n, N = n + 1;
    const size_t es = f->wide ? sizeof(uint64_t) : sizeof(uint32_t);
    int rc = BSW_OK;
    uint8_t *d_ref = nullptr;
    if ((rc = hip_rc(hipSetDevice(f->device))) != BSW_OK) return rc;
    if ((rc = hip_rc(hipMalloc(&f->d_text, (size_t)n + 64))) != BSW_OK) return rc;
    if ((rc = hip_rc(hipMalloc(&f->d_isa, (size_t)N * es))) != BSW_OK) return rc;
    if ((rc = hip_rc(hipMalloc(&d_ref, (size_t)std::max<int64_t>(len, 1)))) != BSW_OK) return rc;
    rc = hip_rc(hipMemcpy(d_ref, ref, (size_t)len, hipMemcpyHostToDevice));
    const unsigned grid = 1u << 16;                      // grid-stride (an AQL grid is 32-bit)
    if (rc == BSW_OK) {
        hipLaunchKernelGGL(k_text_pad, dim3(grid), dim3(256), 0, 0, d_ref, len, f->d_text);
        if (f->wide)
            hipLaunchKernelGGL(k_isa<uint64_t>, dim3(grid), dim3(256), 0, 0, (const uint64_t *)f->d_sa, N,
                               (uint64_t *)f->d_isa);
        else
            hipLaunchKernelGGL(k_isa<uint32_t>, dim3(grid), dim3(256), 0, 0, (const uint32_t *)f->d_sa, N,
                               (uint32_t *)f->d_isa);
        rc = hip_rc(hipGetLastError());
    }
    if (rc == BSW_OK) rc = hip_rc(hipDeviceSynchronize());
    (void)hipFree(d_ref);
    if (rc) return rc;
    f->dev_bytes += (int64_t)n + 64 + N * (int64_t)es;
    if (f->wide) {
        f->dv64.text = f->d_text;
        f->dv64.sa = (const uint64_t *)f->d_sa;
        f->dv64.isa = (const uint64_t *)f->d_isa;
    } else {
        f->dv32.text = f->d_text;
        f->dv32.sa = (const uint32_t *)f->d_sa;
        f->dv32.isa = (const uint32_t *)f->d_isa;
    }
    return BSW_OK;
}

// The k-mer interval table's depth: floor(log4 |T|) - 1 levels (strings that short still occur
// ~4+ times, so the walks would spend their loads on them), at most 15 (22.9 GB of 16-B entries,
// a 3 Gb genome's depth; 13 / 14 / 15 levels measured 314 / 290 / 283 ms of SMEM kernel per 10M
// C4 reads, profiles/r04/ab_smem_ktab.txt); BSW_FMI_KTAB=<levels> overrides (0: off)
int ktab_levels(int64_t n)
{
    int lg = 0;
    while (lg < 31 && ((int64_t)1 << (2 * (lg + 1))) <= n) ++lg;
    int kt = std::min(15, lg - 1);
    if (const char *e = getenv("BSW_FMI_KTAB")) kt = std::min(15, atoi(e));
    return std::max(0, kt);
}

template <class U>
int build_ktab(bsw_fmi_t *f, FmiDevT<U> &dv)
{
    const int kt = ktab_levels(f->n);
    if (kt <= 0) return BSW_OK;
    // ktab_pack keeps k, l and s in 40 bits: an index whose rows pass that runs without the table
    // (every walk then extends base by base), as launch_collect's packed-entry guard does
    if (sizeof(U) == 8 && (uint64_t)f->n + 2 >= (1ull << 40)) return BSW_OK;
    const size_t ents = (size_t)(((1ull << (2 * (kt + 1))) - 4) / 3);   // levels 1 .. kt
    int rc = hip_rc(hipMalloc(&f->d_ktab, ents * sizeof(uint4)));
    if (rc) return rc;
    for (int j = 1; j <= kt && !rc; ++j) {
        const uint64_t cnt = 1ull << (2 * j);
        const unsigned grid = (unsigned)std::min<uint64_t>(1u << 16, (cnt + 255) / 256);
        hipLaunchKernelGGL(ktab_kernel<U>, dim3(grid), dim3(256), 0, f->stream, dv, j, f->d_ktab);
        rc = hip_rc(hipGetLastError());
    }
    if (!rc) rc = hip_rc(hipStreamSynchronize(f->stream));
    if (rc) return rc;
    dv.ktab = f->d_ktab;
    dv.kt = kt;
    f->kt = kt;
    f->dev_bytes += (int64_t)(ents * sizeof(uint4));
    // the counts-only copy (BSW_FMI_STAB=0: off) when every count fits 32 bits: the largest is a
    // single base's (~1.8e9 at 3 Gb)
    int64_t smax = 0;
    for (int c = 0; c < 4; ++c) smax = std::max(smax, f->count[c + 1] - f->count[c]);
    const char *se = getenv("BSW_FMI_STAB");
    if ((se == nullptr || atoi(se) != 0) && smax < ((int64_t)1 << 32)) {
        if (hipMalloc(&f->d_stab, ents * sizeof(uint32_t)) != hipSuccess) {
            (void)hipGetLastError();
            f->d_stab = nullptr;                       // optional: the walks use the full entries
            return BSW_OK;
        }
        const unsigned grid = (unsigned)std::min<uint64_t>(1u << 16, (ents + 255) / 256);
        hipLaunchKernelGGL(stab_kernel, dim3(grid), dim3(256), 0, f->stream, f->d_ktab, (uint64_t)ents, f->d_stab);
        rc = hip_rc(hipGetLastError());
        if (!rc) rc = hip_rc(hipStreamSynchronize(f->stream));
        if (rc) return rc;
        dv.stab = f->d_stab;
        f->dev_bytes += (int64_t)(ents * sizeof(uint32_t));
    }
    return BSW_OK;
}

int finish_device_index(bsw_fmi_t *f)
{
    int rc = BSW_OK;
    if ((rc = hip_rc(hipMalloc(&f->d_err, sizeof(int32_t)))) == BSW_OK &&
        (rc = hip_rc(hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking))) == BSW_OK &&
        (rc = hip_rc(hipEventCreate(&f->ev0))) == BSW_OK && (rc = hip_rc(hipEventCreate(&f->ev1))) == BSW_OK) {
        if (f->wide) {
            f->dv64.blk = f->d_blk;
            for (int c = 0; c < 5; ++c) f->dv64.count[c] = (uint64_t)f->count[c];
            f->dv64.sentinel = (uint64_t)f->sentinel;
            f->dv64.n = (uint64_t)f->n;
        } else {
            f->dv32.blk = f->d_blk;
            for (int c = 0; c < 5; ++c) f->dv32.count[c] = (uint32_t)f->count[c];
            f->dv32.sentinel = (uint32_t)f->sentinel;
            f->dv32.n = (uint32_t)f->n;
        }
    }
    return rc;
}

}  // namespace

extern "C" {

void bsw_mem_opt_default(bsw_mem_opt_t *opt)
{
    opt->min_seed_len = 19;
    opt->split_width = 10;
    opt->max_mem_intv = 20;
    opt->split_factor = 1.5f;
}

int bsw_fmi_build2(const uint8_t *ref, int64_t ref_len, int device, int flags, bsw_fmi_t **out)
{
    if (!out || (!ref && ref_len > 0) || ref_len < 0 || (flags & ~15)) return BSW_E_INVAL;
    const bool text = !(flags & BSW_FMI_NO_TEXT);
    *out = nullptr;
    for (int64_t i = 0; i < ref_len; ++i)
        if (ref[i] > 3) return BSW_E_INVAL;
    const bool need_wide = 2 * ref_len + 2 >= (int64_t)UINT32_MAX;
    const bool wide = need_wide || (flags & BSW_FMI_WIDE);
    const bool gpu = wide || (flags & BSW_FMI_GPU_BUILD) || ref_len >= ((int64_t)64 << 20);
    int ndev = 0;
    if (device >= 0 && (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev)) return BSW_E_NODEV;
    if (gpu && device < 0) return need_wide ? BSW_E_RANGE : BSW_E_INVAL;
    const auto t0 = std::chrono::steady_clock::now();
    if (gpu) {
        bsw::GpuIndex g;
        const int rc = bsw::fmi_build_gpu(ref, ref_len, device, wide, &g);
        if (rc) return rc;
        bsw_fmi_t *f = new bsw_fmi_t;
        f->plain_ent = (flags & BSW_FMI_PLAIN_ENT) != 0;
        f->device = device;
        f->n = g.n;
        f->wide = wide;
        f->gpu_built = true;
        f->d_sa = g.d_sa;
        f->d_blk = g.d_blk;
        f->d_bwt = g.d_bwt;
        f->sentinel = g.sentinel;
        f->tie_groups = g.tie_groups;
        for (int c = 0; c < 5; ++c) f->count[c] = g.count[c];
        const int64_t N = f->n + 1, nb = (N >> 6) + 1;
        f->dev_bytes = nb * 64 + N * (int64_t)(wide ? sizeof(uint64_t) : sizeof(uint32_t)) + N;
        f->build_s = std::chrono::duration<float>(std::chrono::steady_clock::now() - t0).count();
        int r2 = finish_device_index(f);
        if (!r2 && text) r2 = attach_text(f, ref, ref_len);
        if (!r2) r2 = wide ? build_ktab(f, f->dv64) : build_ktab(f, f->dv32);
        if (r2) { bsw_fmi_destroy(f); return r2; }
        f->build_s = std::chrono::duration<float>(std::chrono::steady_clock::now() - t0).count();
        *out = f;
        return BSW_OK;
    }
    const uint32_t n = (uint32_t)(2 * ref_len), N = n + 1;
    std::vector<uint8_t> t(n);
    for (int64_t i = 0; i < ref_len; ++i) {
        t[i] = ref[i];
        t[n - 1 - i] = (uint8_t)(3 - ref[i]);
    }
    bsw_fmi_t *f = new bsw_fmi_t;
    f->plain_ent = (flags & BSW_FMI_PLAIN_ENT) != 0;
    f->device = device;
    f->n = n;
    build_sa(t.data(), n, f->sa);
    f->bwt.resize(N);
    uint32_t sentinel = 0;
    for (uint32_t r = 0; r < N; ++r) {
        const uint32_t p = f->sa[r];
        f->bwt[r] = p == 0 ? 4 : t[p - 1];
        if (p == 0) sentinel = r;
    }
    const size_t nb = (size_t)(N >> 6) + 1;                  // covers row N (= k + s at most)
    std::vector<FmiBlock> blk(nb);
    uint32_t run[4] = {0, 0, 0, 0};
    for (size_t b = 0; b < nb; ++b) {
        FmiBlock &B = blk[b];
        memset(&B, 0, sizeof(B));
        for (int c = 0; c < 4; ++c) B.cnt[c] = run[c];
        for (uint32_t y = 0; y < 64; ++y) {
            const size_t r = b * 64 + y;
            if (r >= N) break;
            const uint8_t c = f->bwt[r];
            if (c < 4) { B.bits[c] |= 1ull << y; run[c]++; }
        }
    }
    f->count[0] = 1;
    for (int c = 0; c < 4; ++c) f->count[c + 1] = f->count[c] + run[c];
    f->build_s = std::chrono::duration<float>(std::chrono::steady_clock::now() - t0).count();
    f->sentinel = sentinel;
    if (device < 0) {                        // host-only index (tests of the builder): no HBM copy
        f->h_blk.swap(blk);
        f->dv32.blk = f->h_blk.data();
        for (int c = 0; c < 5; ++c) f->dv32.count[c] = (uint32_t)f->count[c];
        f->dv32.sentinel = sentinel;
        f->dv32.n = n;
        *out = f;
        return BSW_OK;
    }
    int rc = BSW_OK;
    if ((rc = hip_rc(hipSetDevice(device))) == BSW_OK &&
        (rc = hip_rc(hipMalloc(&f->d_blk, nb * sizeof(FmiBlock)))) == BSW_OK &&
        (rc = hip_rc(hipMalloc(&f->d_sa, (size_t)N * sizeof(uint32_t)))) == BSW_OK &&
        (rc = hip_rc(hipMemcpy(f->d_blk, blk.data(), nb * sizeof(FmiBlock), hipMemcpyHostToDevice))) == BSW_OK &&
        (rc = hip_rc(hipMemcpy(f->d_sa, f->sa.data(), (size_t)N * sizeof(uint32_t), hipMemcpyHostToDevice))) == BSW_OK &&
        (rc = finish_device_index(f)) == BSW_OK) {
        f->dev_bytes = (int64_t)(nb * sizeof(FmiBlock) + (size_t)N * sizeof(uint32_t));
        if ((!text || (rc = attach_text(f, ref, ref_len)) == BSW_OK) && (rc = build_ktab(f, f->dv32)) == BSW_OK) {
            *out = f;
            return BSW_OK;
        }
    }
    bsw_fmi_destroy(f);
    return rc;
}

int bsw_fmi_build(const uint8_t *ref, int64_t ref_len, int device, bsw_fmi_t **out)
{
    return bsw_fmi_build2(ref, ref_len, device, 0, out);
}

void bsw_fmi_destroy(bsw_fmi_t *f)
{
    if (!f) return;
    if (f->device >= 0) (void)hipSetDevice(f->device);
    if (f->d_blk) (void)hipFree(f->d_blk);
    if (f->d_sa) (void)hipFree(f->d_sa);
    if (f->d_bwt) (void)hipFree(f->d_bwt);
    if (f->d_text) (void)hipFree(f->d_text);
    if (f->d_isa) (void)hipFree(f->d_isa);
    if (f->d_ktab) (void)hipFree(f->d_ktab);
    if (f->d_stab) (void)hipFree(f->d_stab);
    if (f->d_err) (void)hipFree(f->d_err);
    if (f->d_scratch) (void)hipFree(f->d_scratch);
    if (f->ev0) (void)hipEventDestroy(f->ev0);
    if (f->ev1) (void)hipEventDestroy(f->ev1);
    if (f->stream) (void)hipStreamDestroy(f->stream);
    delete f;
}

int bsw_fmi_get_info(const bsw_fmi_t *f, bsw_fmi_info_t *out)
{
    if (!f || !out) return BSW_E_INVAL;
    out->n = f->n;
    out->sentinel = f->sentinel;
    for (int c = 0; c < 5; ++c) out->count[c] = f->count[c];
    out->device_bytes = f->dev_bytes;
    out->build_s = f->build_s;
    return BSW_OK;
}

int bsw_fmi_copy_sa(const bsw_fmi_t *f, int64_t *sa)
{
    if (!f || !sa) return BSW_E_INVAL;
    if (!f->gpu_built) {
        for (size_t r = 0; r < f->sa.size(); ++r) sa[r] = f->sa[r];
        return BSW_OK;
    }
    const size_t N = (size_t)f->n + 1;
    if (hipSetDevice(f->device) != hipSuccess) return BSW_E_HIP;
    if (f->wide) return hip_rc(hipMemcpy(sa, f->d_sa, N * sizeof(uint64_t), hipMemcpyDeviceToHost));
    std::vector<uint32_t> t(N);
    const int rc = hip_rc(hipMemcpy(t.data(), f->d_sa, N * sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (size_t r = 0; r < N && !rc; ++r) sa[r] = t[r];
    return rc;
}

int bsw_fmi_check(bsw_fmi_t *f, int64_t *bad)
{
    if (!f || !bad) return BSW_E_INVAL;
    if (f->device < 0) return BSW_E_NODEV;
    std::lock_guard<std::mutex> lk(f->mu);
    if (hipSetDevice(f->device) != hipSuccess) return BSW_E_HIP;
    uint8_t *d_bwt = f->d_bwt;
    bool own = false;
    if (!d_bwt) {                                   // host-built: its BWT codes go up for the check
        if (hipMalloc(&d_bwt, f->bwt.size()) != hipSuccess) return BSW_E_NOMEM;
        own = true;
        if (hipMemcpy(d_bwt, f->bwt.data(), f->bwt.size(), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d_bwt);
            return BSW_E_HIP;
        }
    }
    const int rc = bsw::fmi_check_gpu(f->device, f->wide, f->d_sa, d_bwt, f->d_blk, f->n, f->count, bad);
    if (own) (void)hipFree(d_bwt);
    return rc;
}

int bsw_fmi_copy_bwt(const bsw_fmi_t *f, uint8_t *bwt)
{
    if (!f || !bwt) return BSW_E_INVAL;
    if (!f->gpu_built) {
        memcpy(bwt, f->bwt.data(), f->bwt.size());
        return BSW_OK;
    }
    if (hipSetDevice(f->device) != hipSuccess) return BSW_E_HIP;
    return hip_rc(hipMemcpy(bwt, f->d_bwt, (size_t)f->n + 1, hipMemcpyDeviceToHost));
}

int bsw_mem_collect_intv_device(bsw_fmi_t *f, const bsw_mem_opt_t *opt, const uint8_t *d_reads,
                                const int64_t *d_read_off, const int32_t *d_read_len, int32_t n, int32_t max_len,
                                bsw_bwtintv_t *d_mems, int32_t cap, int32_t *d_n_mems, void *stream)
{
    if (!f || !opt || n < 0 || cap < 0 || max_len < 0 || max_len > BSW_MAX_LEN) return BSW_E_INVAL;
    if (f->device < 0) return BSW_E_NODEV;
    if (n == 0) return BSW_OK;
    if (!d_reads || !d_read_off || !d_read_len || !d_n_mems || (!d_mems && cap > 0)) return BSW_E_INVAL;
    if (opt->min_seed_len < 1 || opt->split_width < 0 || opt->max_mem_intv < 0) return BSW_E_INVAL;
    std::lock_guard<std::mutex> lk(f->mu);
    if (hipSetDevice(f->device) != hipSuccess) return BSW_E_HIP;
    hipStream_t s = stream ? (hipStream_t)stream : f->stream;
    return run_collect(f, opt, d_reads, d_read_off, d_read_len, n, max_len, d_mems, cap, d_n_mems, s);
}

int bsw_mem_collect_intv(bsw_fmi_t *f, const bsw_mem_opt_t *opt, const uint8_t *reads, const int64_t *read_off,
                         const int32_t *read_len, int32_t n, bsw_bwtintv_t *mems, int32_t cap, int32_t *n_mems)
{
    if (!f || !opt || n < 0 || cap < 0) return BSW_E_INVAL;
    if (f->device < 0) return BSW_E_NODEV;
    if (n == 0) return BSW_OK;
    if (!reads || !read_off || !read_len || !n_mems || (!mems && cap > 0)) return BSW_E_INVAL;
    // pack the reads the calls address into one contiguous device buffer
    std::vector<int64_t> off(n);
    int64_t tot = 0;
    int32_t max_len = 0;
    for (int32_t i = 0; i < n; ++i) {
        if (read_len[i] < 0 || read_len[i] > BSW_MAX_LEN || read_off[i] < 0) return BSW_E_RANGE;
        off[i] = tot;
        tot += read_len[i];
        max_len = std::max(max_len, read_len[i]);
    }
    std::vector<uint8_t> buf((size_t)std::max<int64_t>(tot, 1));
    for (int32_t i = 0; i < n; ++i) memcpy(buf.data() + off[i], reads + read_off[i], (size_t)read_len[i]);
    std::lock_guard<std::mutex> lk(f->mu);
    if (hipSetDevice(f->device) != hipSuccess) return BSW_E_HIP;
    uint8_t *d_reads = nullptr;
    int64_t *d_off = nullptr;
    int32_t *d_len = nullptr, *d_cnt = nullptr;
    bsw_bwtintv_t *d_mems = nullptr;
    int rc = BSW_OK;
    hipStream_t s = f->stream;
    if ((rc = hip_rc(hipMalloc(&d_reads, buf.size()))) == BSW_OK &&
        (rc = hip_rc(hipMalloc(&d_off, sizeof(int64_t) * n))) == BSW_OK &&
        (rc = hip_rc(hipMalloc(&d_len, sizeof(int32_t) * n))) == BSW_OK &&
        (rc = hip_rc(hipMalloc(&d_cnt, sizeof(int32_t) * n))) == BSW_OK &&
        (rc = hip_rc(hipMalloc(&d_mems, sizeof(bsw_bwtintv_t) * ((size_t)n * cap + 1)))) == BSW_OK &&
        (rc = hip_rc(hipMemcpyAsync(d_reads, buf.data(), buf.size(), hipMemcpyHostToDevice, s))) == BSW_OK &&
        (rc = hip_rc(hipMemcpyAsync(d_off, off.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, s))) == BSW_OK &&
        (rc = hip_rc(hipMemcpyAsync(d_len, read_len, sizeof(int32_t) * n, hipMemcpyHostToDevice, s))) == BSW_OK) {
        const int krc = run_collect(f, opt, d_reads, d_off, d_len, n, max_len, d_mems, cap, d_cnt, s);
        if (krc == BSW_OK || krc == BSW_E_RANGE) {
            if ((rc = hip_rc(hipMemcpyAsync(n_mems, d_cnt, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s))) == BSW_OK &&
                (cap == 0 || (rc = hip_rc(hipMemcpyAsync(mems, d_mems, sizeof(bsw_bwtintv_t) * (size_t)n * cap,
                                                         hipMemcpyDeviceToHost, s))) == BSW_OK) &&
                (rc = hip_rc(hipStreamSynchronize(s))) == BSW_OK)
                rc = krc;
        } else {
            rc = krc;
        }
    }
    (void)hipStreamSynchronize(s);
    (void)hipFree(d_reads); (void)hipFree(d_off); (void)hipFree(d_len); (void)hipFree(d_cnt); (void)hipFree(d_mems);
    return rc;
}

int bsw_fmi_sa_device(bsw_fmi_t *f, const uint64_t *d_k, int64_t n, int64_t *d_pos, void *stream)
{
    if (!f || n < 0 || (n > 0 && (!d_k || !d_pos))) return BSW_E_INVAL;
    if (f->device < 0) return BSW_E_NODEV;
    if (n == 0) return BSW_OK;
    if (hipSetDevice(f->device) != hipSuccess) return BSW_E_HIP;
    hipStream_t s = stream ? (hipStream_t)stream : f->stream;
    if (f->wide)
        hipLaunchKernelGGL(sa_kernel<uint64_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                           (const uint64_t *)f->d_sa, (uint64_t)f->n + 1, d_k, n, d_pos);
    else
        hipLaunchKernelGGL(sa_kernel<uint32_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                           (const uint32_t *)f->d_sa, (uint64_t)f->n + 1, d_k, n, d_pos);
    if (hipGetLastError() != hipSuccess) return BSW_E_HIP;
    return hipStreamSynchronize(s) == hipSuccess ? BSW_OK : BSW_E_HIP;
}

int bsw_fmi_last_kernel_ms(const bsw_fmi_t *f, float *ms)
{
    if (!f || !ms) return BSW_E_INVAL;
    *ms = f->kernel_ms;
    return BSW_OK;
}

}  // extern "C"

