/* bsw_batch.c -- ".bswb" batch files (include/bsw_batch.h): record / replay of SeqPair
 * batches.  Plain C stdio, no device code. */
#include <stdio.h>
#include <string.h>
#include "../../include/bsw_batch.h"

_Static_assert(sizeof(bswb_header_t) == 128, "bswb header is 128 bytes");

static uint64_t fnv1a(uint64_t h, const void *p, size_t n)
{
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001B3ull; }
    return h;
}
#define FNV0 0xCBF29CE484222325ull

int bswb_write(const char *path, const bsw_params_t *params, int32_t w, int32_t cell_bits,
               int has_outputs, const SeqPair *pairs, int64_t n_pairs, const uint8_t *ref,
               int64_t ref_bytes, const uint8_t *qer, int64_t qer_bytes)
{
    if (!path || !params || n_pairs < 0 || ref_bytes < 0 || qer_bytes < 0 ||
        (n_pairs && !pairs) || (ref_bytes && !ref) || (qer_bytes && !qer))
        return BSW_E_INVAL;
    bswb_header_t h;
    memset(&h, 0, sizeof(h));
    h.magic = BSWB_MAGIC; h.version = BSWB_VERSION; h.header_bytes = sizeof(h);
    h.flags = has_outputs ? BSWB_HAS_OUTPUTS : 0u;
    h.n_pairs = n_pairs; h.ref_bytes = ref_bytes; h.qer_bytes = qer_bytes;
    h.w = w; h.cell_bits = cell_bits; h.params = *params;
    uint64_t c = FNV0;
    c = fnv1a(c, pairs, (size_t)n_pairs * sizeof(SeqPair));
    c = fnv1a(c, ref, (size_t)ref_bytes);
    c = fnv1a(c, qer, (size_t)qer_bytes);
    h.checksum = c;
    FILE *f = fopen(path, "wb");
    if (!f) return BSW_E_INVAL;
    int ok = fwrite(&h, sizeof(h), 1, f) == 1;
    if (ok && n_pairs) ok = fwrite(pairs, sizeof(SeqPair), (size_t)n_pairs, f) == (size_t)n_pairs;
    if (ok && ref_bytes) ok = fwrite(ref, 1, (size_t)ref_bytes, f) == (size_t)ref_bytes;
    if (ok && qer_bytes) ok = fwrite(qer, 1, (size_t)qer_bytes, f) == (size_t)qer_bytes;
    ok = (fclose(f) == 0) && ok;
    return ok ? BSW_OK : BSW_E_INVAL;
}

int bswb_read_header(const char *path, bswb_header_t *h)
{
    if (!path || !h) return BSW_E_INVAL;
    FILE *f = fopen(path, "rb");
    if (!f) return BSW_E_INVAL;
    int ok = fread(h, sizeof(*h), 1, f) == 1;
    long long len = -1;
    if (ok && fseek(f, 0, SEEK_END) == 0) len = ftell(f);
    fclose(f);
    if (!ok || h->magic != BSWB_MAGIC || h->version != BSWB_VERSION || h->header_bytes != sizeof(*h))
        return BSW_E_INVAL;
    if (h->n_pairs < 0 || h->ref_bytes < 0 || h->qer_bytes < 0) return BSW_E_RANGE;
    const long long want = (long long)sizeof(*h) + h->n_pairs * (long long)sizeof(SeqPair) +
                           h->ref_bytes + h->qer_bytes;
    if (len != want) return BSW_E_RANGE;
    return BSW_OK;
}

int bswb_read(const char *path, bswb_header_t *h, SeqPair *pairs, uint8_t *ref, uint8_t *qer)
{
    int rc = bswb_read_header(path, h);
    if (rc) return rc;
    if ((h->n_pairs && !pairs) || (h->ref_bytes && !ref) || (h->qer_bytes && !qer)) return BSW_E_INVAL;
    FILE *f = fopen(path, "rb");
    if (!f) return BSW_E_INVAL;
    int ok = fseek(f, (long)sizeof(*h), SEEK_SET) == 0;
    if (ok && h->n_pairs) ok = fread(pairs, sizeof(SeqPair), (size_t)h->n_pairs, f) == (size_t)h->n_pairs;
    if (ok && h->ref_bytes) ok = fread(ref, 1, (size_t)h->ref_bytes, f) == (size_t)h->ref_bytes;
    if (ok && h->qer_bytes) ok = fread(qer, 1, (size_t)h->qer_bytes, f) == (size_t)h->qer_bytes;
    fclose(f);
    if (!ok) return BSW_E_RANGE;
    uint64_t c = FNV0;
    c = fnv1a(c, pairs, (size_t)h->n_pairs * sizeof(SeqPair));
    c = fnv1a(c, ref, (size_t)h->ref_bytes);
    c = fnv1a(c, qer, (size_t)h->qer_bytes);
    return c == h->checksum ? BSW_OK : BSW_E_RANGE;
}
