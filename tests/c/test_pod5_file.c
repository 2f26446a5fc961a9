/* test_pod5_file.c -- a C program against include/pgnano_pod5file.h, linked with libpgnano_hip.so
 * (test infrastructure): `copy in.pod5 mid.pod5 --pgnano` then `copy mid.pod5 out.pod5 --VBZ` through
 * pgn_pod5_transcode_file, the double-conversion protocol of the reference's integration check
 * (test_scripts/double_conversion.py:37-69).  The VBZ signal column that comes back must equal the
 * input's byte for byte (the GPU VBZ encoder writes the pod5 writer's frames), the read ids and
 * sample counts must be unchanged, and every other embedded table must be the input's bytes.
 * Usage: test_pod5_file IN.pod5 WORKDIR.  Exit 0: pass; 77: no HIP device (skipped); else failure. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pgnano_pod5file.h"
#include "pgnano_pod5.h"

typedef struct {
    uint64_t rows, bytes, samples;
    uint32_t batches;
    int type;
    uint8_t *ids, *data;
    uint32_t *cnt;
    uint64_t *offs;
} table_t;

static int load(const char *path, pgn_pod5_file **f, table_t *t)
{
    int rc = pgn_pod5_file_open(path, f);
    if (rc) {
        fprintf(stderr, "open %s: %s (%s)\n", path, pgn_status_string(rc), pgn_pod5_file_error());
        return rc;
    }
    pgn_pod5_signal_info(*f, &t->rows, &t->batches, &t->type, &t->bytes, &t->samples);
    t->ids = (uint8_t *)malloc(16 * t->rows + 1);
    t->data = (uint8_t *)malloc(t->bytes + 1);
    t->cnt = (uint32_t *)malloc(4 * t->rows + 4);
    t->offs = (uint64_t *)malloc(8 * (t->rows + 1));
    return pgn_pod5_signal_read(*f, t->ids, t->cnt, t->offs, t->data);
}

static void release(pgn_pod5_file *f, table_t *t)
{
    free(t->ids);
    free(t->data);
    free(t->cnt);
    free(t->offs);
    pgn_pod5_file_close(f);
}

static int same_tables(const pgn_pod5_file *a, const pgn_pod5_file *b, FILE *fa, FILE *fb)
{
    /* every non-signal table of a appears in b with the same bytes */
    for (int i = 0; i < pgn_pod5_file_embedded_count(a); i++) {
        int64_t oa, la, ob, lb;
        int ta, tb;
        pgn_pod5_file_embedded(a, i, &oa, &la, &ta);
        if (ta == PGN_POD5_CONTENT_SIGNAL) continue;
        int found = 0;
        for (int j = 0; j < pgn_pod5_file_embedded_count(b); j++) {
            pgn_pod5_file_embedded(b, j, &ob, &lb, &tb);
            if (tb != ta) continue;
            found = 1;
            if (la != lb) return 0;
            char *x = (char *)malloc((size_t)la + 1), *y = (char *)malloc((size_t)lb + 1);
            fseek(fa, (long)oa, SEEK_SET);
            fseek(fb, (long)ob, SEEK_SET);
            const int ok = fread(x, 1, (size_t)la, fa) == (size_t)la && fread(y, 1, (size_t)lb, fb) == (size_t)lb &&
                           memcmp(x, y, (size_t)la) == 0;
            free(x);
            free(y);
            if (!ok) return 0;
        }
        if (!found) return 0;
    }
    return 1;
}

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s IN.pod5 WORKDIR\n", argv[0]);
        return 2;
    }
    char mid[4096], out[4096];
    snprintf(mid, sizeof(mid), "%s/mid_pgnano.pod5", argv[2]);
    snprintf(out, sizeof(out), "%s/back_vbz.pod5", argv[2]);
    pgn_ctx *ctx = NULL;
    int rc = pgn_ctx_create(0, &ctx);
    if (rc == PGN_ERR_NO_DEVICE) {
        printf("no HIP device: skipped\n");
        return 77;
    }
    if (rc) {
        fprintf(stderr, "ctx: %s\n", pgn_status_string(rc));
        return 1;
    }
    pgn_pod5_transcode_stats s1, s2;
    rc = pgn_pod5_transcode_file(ctx, argv[1], mid, PGN_POD5_SIGNAL_PGNANO, PGN_VARIANT_C5, 0, &s1);
    if (rc) {
        fprintf(stderr, "--pgnano: %s (%s)\n", pgn_status_string(rc), pgn_pod5_last_error());
        return 1;
    }
    rc = pgn_pod5_transcode_file(ctx, mid, out, PGN_POD5_SIGNAL_VBZ, PGN_VARIANT_C5, 0, &s2);
    if (rc) {
        fprintf(stderr, "--VBZ: %s (%s)\n", pgn_status_string(rc), pgn_pod5_last_error());
        return 1;
    }
    pgn_pod5_file *fi, *fm, *fo;
    table_t ti, tm, to;
    if (load(argv[1], &fi, &ti) || load(mid, &fm, &tm) || load(out, &fo, &to)) return 1;
    int ok = tm.type == PGN_POD5_SIGNAL_PGNANO && to.type == ti.type && to.rows == ti.rows && tm.rows == ti.rows;
    ok = ok && to.bytes == ti.bytes && memcmp(to.data, ti.data, ti.bytes) == 0;
    ok = ok && memcmp(to.offs, ti.offs, 8 * (ti.rows + 1)) == 0 && memcmp(to.cnt, ti.cnt, 4 * ti.rows) == 0;
    ok = ok && memcmp(tm.ids, ti.ids, 16 * ti.rows) == 0 && memcmp(to.ids, ti.ids, 16 * ti.rows) == 0;
    ok = ok && strcmp(pgn_pod5_file_identifier(fo), pgn_pod5_file_identifier(fi)) == 0;
    FILE *a = fopen(argv[1], "rb"), *b = fopen(out, "rb");
    ok = ok && a && b && same_tables(fi, fo, a, b);
    if (a) fclose(a);
    if (b) fclose(b);
    printf("rows %llu samples %llu: vbz %llu B -> pgnano %llu B (%.4f bits/sample, encode %.3f ms) -> vbz %llu B: %s\n",
           (unsigned long long)s1.rows, (unsigned long long)s1.samples, (unsigned long long)s1.in_bytes,
           (unsigned long long)s1.out_bytes, 8.0 * (double)s1.out_bytes / (double)(s1.samples ? s1.samples : 1),
           s1.encode_ms, (unsigned long long)s2.out_bytes, ok ? "identical" : "MISMATCH");
    release(fi, &ti);
    release(fm, &tm);
    release(fo, &to);
    pgn_ctx_destroy(ctx);
    return ok ? 0 : 1;
}
