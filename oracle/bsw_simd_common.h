/* oracle/bsw_simd_common.h -- shared declarations of the CPU baseline (bsw_sse41.c, bsw_avx512.c) */
#ifndef BSW_SIMD_COMMON_H
#define BSW_SIMD_COMMON_H
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../include/bsw_seqpair.h"

#define DUMMY1 99
#define DUMMY2 100

typedef struct {
    int32_t o_del, e_del, o_ins, e_ins, zdrop, end_bonus;
    int8_t mat[25];
} sse_params_t;

int oracle_ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target,
                       int m, const int8_t *mat, int o_del, int e_del, int o_ins,
                       int e_ins, int w, int end_bonus, int zdrop, int h0, int *_qle,
                       int *_tle, int *_gtle, int *_gscore, int *_max_off);

static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int imin(int a, int b) { return a < b ? a : b; }

typedef struct {
    const sse_params_t *p;
    SeqPair **order;
    int32_t n, w, maxsc;
    const uint8_t *ref, *qer;
    volatile int32_t *next;
} simd_job_t;

/* per-lane band cap (A.2), integer form of (int)((double)N / e + 1.) */
static int band_cap(const sse_params_t *p, int qlen, int w, int maxsc)
{
    int n_ins = qlen * maxsc + p->end_bonus - p->o_ins;
    int n_del = qlen * maxsc + p->end_bonus - p->o_del;
    int mi = (n_ins + p->e_ins) / p->e_ins, md = (n_del + p->e_del) / p->e_del;
    mi = mi > 1 ? mi : 1;
    md = md > 1 ? md : 1;
    w = w < mi ? w : mi;
    return w < md ? w : md;
}

#endif
