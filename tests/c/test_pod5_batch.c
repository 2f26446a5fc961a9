/* test_pod5_batch.c -- a C program compiled against include/pgnano_pod5.h and include/pgnano_hip.h
 * and linked with libpgnano_hip.so, as a C/C++ POD5 writer/reader would use them (test
 * infrastructure).  A pod5_add_reads_data-shaped batch (reads of different lengths, one above two
 * writer chunks) is compressed in one call; every chunk must equal the per-chunk plugin entry point's
 * bytes (pgn_compress_signal / pgn_vbz_compress_signal -- the drop-in path the reference calls once
 * per chunk), and the rows must decode back to the reads through pgn_pod5_decompress_rows.
 * Exit 0: pass; 77: no HIP device (skipped); anything else: failure. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pgnano_pod5.h"

static uint64_t mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* nanopore-like: piecewise-constant levels plus small noise */
static void make_read(int16_t *x, uint32_t n, uint64_t seed)
{
    int32_t level = 500;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t r = mix(seed * 0x9E3779B97F4A7C15ull + i);
        if ((r & 15) == 0) level = 350 + (int32_t)((r >> 8) % 300);
        x[i] = (int16_t)(level + (int32_t)((r >> 20) % 41) - 20);
    }
}

static int run(pgn_ctx *ctx, int codec, uint32_t chunk)
{
    enum { READS = 7 };
    const uint32_t len[READS] = {100000, 0, 1, 250000, 102400, 37, 204801};
    int16_t *sig[READS];
    for (int r = 0; r < READS; r++) {
        sig[r] = (int16_t *)malloc(2 * (size_t)(len[r] ? len[r] : 1));
        make_read(sig[r], len[r], 1000 + r);
    }
    pgn_pod5_batch *b = NULL;
    int rc = pgn_pod5_batch_create(ctx, codec, chunk, &b);
    if (rc) { fprintf(stderr, "create: %d\n", rc); return 1; }
    size_t nchunks = 0;
    const uint64_t *offs;
    const uint8_t *data;
    const uint32_t *samples, *read_index;
    rc = pgn_pod5_compress_reads(b, READS, (const int16_t *const *)sig, len, &nchunks, &offs, &data, &samples, &read_index);
    if (rc) { fprintf(stderr, "compress_reads: %d (%s)\n", rc, pgn_status_string(rc)); return 1; }
    /* the writer's chunking: ceil(n / chunk) chunks per read, in read order */
    const uint32_t cs = chunk ? chunk : PGN_POD5_DEFAULT_CHUNK_SIZE;
    size_t want = 0;
    for (int r = 0; r < READS; r++) want += (len[r] + cs - 1) / cs;
    if (nchunks != want) { fprintf(stderr, "chunks %zu != %zu\n", nchunks, want); return 1; }
    /* every chunk = the per-chunk entry point's blob */
    size_t i = 0;
    uint64_t total = 0;
    for (int r = 0; r < READS; r++) {
        for (uint32_t s = 0; s < len[r]; s += cs, i++) {
            const uint32_t n = len[r] - s < cs ? len[r] - s : cs;
            if (read_index[i] != (uint32_t)r || samples[i] != n) { fprintf(stderr, "chunk %zu: read/samples\n", i); return 1; }
            const size_t cap = codec == PGN_POD5_CODEC_VBZ ? pgn_vbz_compressed_signal_max_size(n)
                                                           : pgn_compressed_signal_max_size(n);
            uint8_t *blob = (uint8_t *)malloc(cap);
            size_t sz = 0;
            const int rc1 = codec == PGN_POD5_CODEC_VBZ ? pgn_vbz_compress_signal(ctx, sig[r] + s, n, blob, cap, &sz)
                                                        : pgn_variant_compress_signal(ctx, codec, sig[r] + s, n, blob, cap, &sz);
            if (rc1 || sz != offs[i + 1] - offs[i] || memcmp(blob, data + offs[i], sz) != 0) {
                fprintf(stderr, "chunk %zu: differs from the per-chunk blob (rc %d, %zu vs %llu)\n", i, rc1, sz,
                        (unsigned long long)(offs[i + 1] - offs[i]));
                return 1;
            }
            free(blob);
            total += n;
        }
    }
    /* the reader side: decode the rows back */
    int16_t *back = (int16_t *)malloc(2 * (size_t)total + 2);
    int32_t *st = (int32_t *)malloc(4 * nchunks + 4);
    rc = pgn_pod5_decompress_rows(b, (uint32_t)nchunks, offs, data, samples, back, st);
    if (rc) { fprintf(stderr, "decompress_rows: %d\n", rc); return 1; }
    uint64_t at = 0;
    for (int r = 0; r < READS; r++) {
        if (len[r] && memcmp(back + at, sig[r], 2 * (size_t)len[r]) != 0) { fprintf(stderr, "read %d differs\n", r); return 1; }
        at += len[r];
    }
    printf("codec %d chunk %u: %zu chunks, %llu samples, %llu bytes ok\n", codec, cs, nchunks,
           (unsigned long long)total, (unsigned long long)offs[nchunks]);
    pgn_pod5_batch_destroy(b);
    for (int r = 0; r < READS; r++) free(sig[r]);
    free(back);
    free(st);
    return 0;
}

int main(void)
{
    pgn_ctx *ctx = NULL;
    int rc = pgn_ctx_create(0, &ctx);
    if (rc == PGN_ERR_NO_DEVICE) { printf("no HIP device: skipped\n"); return 77; }
    if (rc) { fprintf(stderr, "ctx: %d\n", rc); return 1; }
    if (run(ctx, PGN_VARIANT_C5, 0) || run(ctx, PGN_POD5_CODEC_VBZ, 0) || run(ctx, PGN_VARIANT_C5, 65536) ||
        run(ctx, PGN_VARIANT_C4, 0))
        return 1;
    pgn_ctx_destroy(ctx);
    printf("pod5 batch: ok\n");
    return 0;
}
