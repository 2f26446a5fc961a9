/*
 * pgn_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the reference's pgnano "C5" codec (COMPRESSOR_C5, the variant
 * compiled by default: pod5/c++/pod5_format/pgnano/pgnano.cpp:1) and of the VBZ codec
 * (pod5/c++/pod5_format/signal_compression.cpp:37-156), both calling the real third-party
 * entropy stage the reference calls: libzstd (ZSTD_compress level 1 / ZSTD_decompress).
 *
 * libzstd is not vendored in the reference (conda `zstd`, unversioned: conda_build:7,
 * install_dependencies.sh:10; pod5/c++/CMakeLists.txt:18 find_package(zstd)).  This image ships
 * libzstd 1.4.9 (/opt/conda/lib) and 1.4.8 (system); it is dlopen()ed here, 1.4.9 first.
 *
 * The whole reference codec is not buildable in this image (the pgnano:: compress/decompress bodies
 * pull BAM_handler.h -> boost + htslib, and pod5_format_export.h is CMake-generated).  Its svb16
 * split/merge stage IS: oracle/ref.mk compiles the `namespace svb16` block of every variant header
 * (C5, C4, C3, C2, C1, VBZ_0) and the pod5 VBZ svb16 stage verbatim from /root/reference into
 * oracle/_ref/, and tests/test_oracle_ref.py holds this restatement's split streams, merge outputs and
 * consumed counts (pgno_variant_streams / pgno_variant_merge / pgno_vbz_svb_encode) to it on the
 * reference fixture, edge sizes, stress and fuzz inputs.  The frame assembly around it (u64 length
 * prefixes, ZSTD_compress level 1, content-size bookkeeping) is pinned by the reference's own VBZ
 * fixture blobs and by reading C5.hpp:282-683 line by line.  See DESIGN.md "Oracle and parity".
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 */
#include <dlfcn.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PGNO_OK 0
#define PGNO_ERR_DST_TOO_SMALL 1   /* "Not enough space in destination buffer"      C5.hpp:420-427 */
#define PGNO_ERR_NOT_ZSTD 2        /* "Input data not compressed by zstd"           C5.hpp:495-502 */
#define PGNO_ERR_ZSTD_DECOMPRESS 3 /* "Input data failed to decompress using zstd"  C5.hpp:593-600 */
#define PGNO_ERR_REMAINING 4       /* "Remaining data at end of signal buffer"      C5.hpp:675-677 */
#define PGNO_ERR_ZSTD_COMPRESS 5   /* "Failed to compress ..."                       C5.hpp:340-342 */
#define PGNO_ERR_CORRUPT 6         /* input the reference would read out of bounds (UB there) */
#define PGNO_ERR_NO_ZSTD 7         /* libzstd could not be loaded */
#define PGNO_ERR_ALLOC 8

/* ----------------------------------------------------------------------------------------------
 * libzstd entry points (the six prototypes the reference uses; zstd.h is not in the repo)
 * -------------------------------------------------------------------------------------------- */
typedef size_t (*fn_compress)(void *, size_t, const void *, size_t, int);
typedef size_t (*fn_decompress)(void *, size_t, const void *, size_t);
typedef unsigned long long (*fn_fcs)(const void *, size_t);
typedef size_t (*fn_bound)(size_t);
typedef unsigned (*fn_iserror)(size_t);
typedef unsigned (*fn_version)(void);

static struct {
    int loaded;
    void *h;
    fn_compress compress;
    fn_decompress decompress;
    fn_fcs fcs;
    fn_bound bound;
    fn_iserror iserror;
    fn_version version;
    char path[512];
} Z;

int pgno_zstd_load(const char *path)
{
    const char *cands[4];
    int nc = 0;
    if (path && path[0]) cands[nc++] = path;
    if (!path || !path[0]) {
        const char *env = getenv("PGN_LIBZSTD");
        if (env && env[0]) cands[nc++] = env;
        cands[nc++] = "/opt/conda/lib/libzstd.so.1.4.9";
        cands[nc++] = "libzstd.so.1";
    }
    if (Z.loaded && !(path && path[0])) return PGNO_OK;
    for (int i = 0; i < nc; i++) {
        void *h = dlopen(cands[i], RTLD_NOW | RTLD_LOCAL);
        if (!h) continue;
        fn_compress c = (fn_compress)dlsym(h, "ZSTD_compress");
        fn_decompress d = (fn_decompress)dlsym(h, "ZSTD_decompress");
        fn_fcs f = (fn_fcs)dlsym(h, "ZSTD_getFrameContentSize");
        fn_bound b = (fn_bound)dlsym(h, "ZSTD_compressBound");
        fn_iserror e = (fn_iserror)dlsym(h, "ZSTD_isError");
        fn_version v = (fn_version)dlsym(h, "ZSTD_versionNumber");
        if (!c || !d || !f || !b || !e || !v) { dlclose(h); continue; }
        Z.h = h; Z.compress = c; Z.decompress = d; Z.fcs = f; Z.bound = b; Z.iserror = e;
        Z.version = v;
        strncpy(Z.path, cands[i], sizeof(Z.path) - 1);
        Z.loaded = 1;
        return PGNO_OK;
    }
    return PGNO_ERR_NO_ZSTD;
}

static int zok(void) { return Z.loaded || pgno_zstd_load(NULL) == PGNO_OK; }

unsigned pgno_zstd_version(void) { return zok() ? Z.version() : 0u; }
const char *pgno_zstd_path(void) { return zok() ? Z.path : ""; }

size_t pgno_zstd_bound(size_t n) { return zok() ? Z.bound(n) : 0; }

/* ZSTD_compress(dst, ZSTD_compressBound(len), src, len, 1), as at C5.hpp:337-339. Returns size or
 * (size_t)-1 on error. */
size_t pgno_zstd_compress1(const uint8_t *src, size_t n, uint8_t *dst, size_t cap)
{
    if (!zok()) return (size_t)-1;
    size_t r = Z.compress(dst, cap, src, n, 1);
    return Z.iserror(r) ? (size_t)-1 : r;
}

/* Frames from other encoder settings, for decoder coverage only (the reference itself always
 * writes level 1).  window_log == 0: ZSTD_compress at `level`.  window_log > 0: the advanced API
 * with ZSTD_c_windowLog forced, which splits the input into blocks of 1 << window_log bytes
 * (multi-block frames: repeat-mode tables, offsets reaching into earlier blocks) and writes a
 * window descriptor instead of a single-segment header. */
typedef void *(*fn_cctx_new)(void);
typedef size_t (*fn_cctx_free)(void *);
typedef size_t (*fn_cctx_set)(void *, int, int);
typedef size_t (*fn_compress2)(void *, void *, size_t, const void *, size_t);
size_t pgno_zstd_compress_ex(const uint8_t *src, size_t n, uint8_t *dst, size_t cap, int level, int window_log)
{
    if (!zok()) return (size_t)-1;
    if (window_log == 0) {
        size_t r = Z.compress(dst, cap, src, n, level);
        return Z.iserror(r) ? (size_t)-1 : r;
    }
    fn_cctx_new cnew = (fn_cctx_new)dlsym(Z.h, "ZSTD_createCCtx");
    fn_cctx_free cfree = (fn_cctx_free)dlsym(Z.h, "ZSTD_freeCCtx");
    fn_cctx_set cset = (fn_cctx_set)dlsym(Z.h, "ZSTD_CCtx_setParameter");
    fn_compress2 c2 = (fn_compress2)dlsym(Z.h, "ZSTD_compress2");
    if (!cnew || !cfree || !cset || !c2) return (size_t)-1;
    void *cc = cnew();
    if (!cc) return (size_t)-1;
    size_t r = cset(cc, 100 /* ZSTD_c_compressionLevel */, level);
    if (!Z.iserror(r)) r = cset(cc, 101 /* ZSTD_c_windowLog */, window_log);
    if (!Z.iserror(r)) r = cset(cc, 200 /* ZSTD_c_contentSizeFlag */, 1);
    if (!Z.iserror(r)) r = c2(cc, dst, cap, src, n);
    cfree(cc);
    return Z.iserror(r) ? (size_t)-1 : r;
}

size_t pgno_zstd_decompress(const uint8_t *src, size_t n, uint8_t *dst, size_t cap)
{
    if (!zok()) return (size_t)-1;
    size_t r = Z.decompress(dst, cap, src, n);
    return Z.iserror(r) ? (size_t)-1 : r;
}

/* Returns content size, or (uint64)-1 when ZSTD_isError() holds for the result (the reference's
 * test, which also catches CONTENTSIZE_UNKNOWN / CONTENTSIZE_ERROR). */
unsigned long long pgno_zstd_content_size(const uint8_t *src, size_t n)
{
    if (!zok()) return (unsigned long long)-1;
    unsigned long long r = Z.fcs(src, n);
    return Z.iserror((size_t)r) ? (unsigned long long)-1 : r;
}

/* ----------------------------------------------------------------------------------------------
 * Shared helpers
 * -------------------------------------------------------------------------------------------- */

/* zig-zag of a wrapping 16-bit delta: pgnano/svb16/encode_scalar.hpp:16-19 */
static inline uint16_t zz_enc(uint16_t v) { return (uint16_t)((uint16_t)(v + v) ^ (uint16_t)((int16_t)v >> 15)); }
/* inverse: pgnano/svb16/decode_scalar.hpp:14-17 */
static inline uint16_t zz_dec(uint16_t v) { return (uint16_t)((v >> 1) ^ (uint16_t)(0u - (v & 1u))); }

/* Plugin output bound: pgnano::Compressor::compressed_signal_max_size (compressor.h:39-45), used by
 * pgnano::compress_signal (pgnano.cpp:66-68): max(2n + header_size(10) + overflow(16), 1024). */
size_t pgno_c5_bound(uint32_t n)
{
    size_t s = (size_t)n * 2u + 10u + 16u;
    return s > 1024u ? s : 1024u;
}

/* Reusable per-thread scratch: the reference allocates from an arrow::MemoryPool (jemalloc), which
 * recycles these buffers between chunks; fresh malloc/mmap per call would time page faults. */
static __thread uint8_t *tl_buf[2];
static __thread size_t tl_cap[2];
static uint8_t *scratch(int i, size_t n)
{
    if (tl_cap[i] < n) {
        free(tl_buf[i]);
        tl_buf[i] = (uint8_t *)malloc(n);
        tl_cap[i] = tl_buf[i] ? n : 0;
    }
    return tl_buf[i];
}

static inline void put_u64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); } /* host-endian size_t */
static inline uint64_t get_u64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

/* ----------------------------------------------------------------------------------------------
 * C5 split: svb16::encode_scalar_N01<int16_t, true, true> (C5.hpp:57-152), prev = 0.
 * keys: 2-bit codes, sample i in bits 2*(i%4) of byte i/4; code 0: v==0; 1: v in [1,16] -> nibble
 * v-1 in S (low nibble first); 2: v in [17,272] -> byte v-17 in M; 3: v>=273 -> w=v-273, Llow=w&255,
 * Lhigh=w>>8.  sizes = {keys, S, M, Llow, Lhigh}.
 * -------------------------------------------------------------------------------------------- */
void pgno_c5_split(const int16_t *x, uint32_t n, uint8_t *keys, uint8_t *S, uint8_t *M,
                   uint8_t *Ll, uint8_t *Lh, uint64_t sizes[5])
{
    if (n == 0) { for (int i = 0; i < 5; i++) sizes[i] = 0; return; }
    uint64_t nk = (n + 3u) / 4u, ns = 0, nm = 0, nl = 0;
    memset(keys, 0, nk);
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint16_t cur = (uint16_t)x[i];
        uint16_t v = zz_enc((uint16_t)(cur - prev));
        prev = cur;
        unsigned code;
        if (v == 0) {
            code = 0;
        } else if (v <= 16) {
            code = 1;
            unsigned nib = (unsigned)(v - 1);
            if ((ns & 1u) == 0) S[ns >> 1] = (uint8_t)nib;
            else S[ns >> 1] |= (uint8_t)(nib << 4);
            ns++;
        } else if (v <= 272) {
            code = 2;
            M[nm++] = (uint8_t)(v - 17);
        } else {
            code = 3;
            unsigned w = (unsigned)v - 273u;
            Ll[nl] = (uint8_t)(w & 0xFFu);
            Lh[nl] = (uint8_t)(w >> 8);
            nl++;
        }
        keys[i >> 2] |= (uint8_t)(code << (2u * (i & 3u)));
    }
    sizes[0] = nk;
    sizes[1] = (ns + 1) / 2;
    sizes[2] = nm;
    sizes[3] = nl;
    sizes[4] = nl;
}

/* C5 merge over the reference's concatenated intermediate (decode_N01 C5.hpp:260-275 ->
 * decode_scalar_N01 C5.hpp:173-257).  Stream starts are keys_length = ceil(n/4) (svb16.h:18-22),
 * then the decompressed sizes dS, dM, dLl of frames 2..4.  Reads go through the concatenated buffer
 * exactly like the reference's pointer walk (a short stream reads into the next one); a read past
 * the end of the buffer (UB in the reference) is reported as PGNO_ERR_CORRUPT.  Returns the
 * consumed count (one past the last Lhigh byte read) through *consumed. */
static int c5_merge(const uint8_t *inter, uint64_t total, uint64_t dS, uint64_t dM, uint64_t dLl,
                    int16_t *out, uint32_t n, uint64_t *consumed)
{
    uint64_t kl = ((uint64_t)n + 3u) / 4u;
    uint64_t ps = kl, pm = kl + dS, pl = kl + dS + dM, ph = kl + dS + dM + dLl;
    if (n == 0) { *consumed = ph; return PGNO_OK; }
    uint64_t sn = 0; /* nibbles consumed */
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t kb = i >> 2;
        if (kb >= total) return PGNO_ERR_CORRUPT;
        unsigned code = (inter[kb] >> (2u * (i & 3u))) & 3u;
        uint16_t v;
        if (code == 0) {
            v = 0;
        } else if (code == 1) {
            uint64_t b = ps + (sn >> 1);
            if (b >= total) return PGNO_ERR_CORRUPT;
            v = (uint16_t)(((sn & 1u) ? (inter[b] >> 4) : (inter[b] & 0xFu)) + 1u);
            sn++;
        } else if (code == 2) {
            if (pm >= total) return PGNO_ERR_CORRUPT;
            v = (uint16_t)(inter[pm++] + 17u);
        } else {
            if (pl >= total || ph >= total) return PGNO_ERR_CORRUPT;
            v = (uint16_t)(((unsigned)inter[ph++] << 8) + inter[pl++] + 273u);
        }
        prev = (uint16_t)(zz_dec(v) + prev);
        out[i] = (int16_t)prev;
    }
    *consumed = ph;
    return PGNO_OK;
}

/* ----------------------------------------------------------------------------------------------
 * C5 compress: compress_signal_N01 (C5.hpp:282-474) behind pgnano::compress_signal (pgnano.cpp:59-96).
 * dst/cap is the caller's destination span (the plugin passes pgno_c5_bound(n) bytes).
 * Wire format: [u64 cK][K][u64 cS][S][u64 cM][M][u64 cLl][Ll][Lh] (C5.hpp:429-462).
 * stream_sizes (optional, 10 entries): raw sizes of the 5 streams then their frame sizes.
 * -------------------------------------------------------------------------------------------- */
int pgno_c5_compress(const int16_t *x, uint32_t n, uint8_t *dst, size_t cap, size_t *out_len,
                     uint64_t *stream_sizes)
{
    if (!zok()) return PGNO_ERR_NO_ZSTD;
    size_t nk = ((size_t)n + 3u) / 4u;
    uint8_t *buf = scratch(0, nk + 4 * (size_t)n + 16);
    if (!buf) return PGNO_ERR_ALLOC;
    uint8_t *st[5];
    st[0] = buf;
    st[1] = st[0] + nk;
    st[2] = st[1] + n;
    st[3] = st[2] + n;
    st[4] = st[3] + n;
    uint64_t sz[5];
    pgno_c5_split(x, n, st[0], st[1], st[2], st[3], st[4], sz);

    uint8_t *fr[5];
    size_t fsz[5], fb[5], ftot = 0;
    int rc = PGNO_OK;
    for (int s = 0; s < 5; s++) { fb[s] = Z.bound(sz[s]); ftot += fb[s]; }
    uint8_t *fbuf = scratch(1, ftot + 16);
    if (!fbuf) return PGNO_ERR_ALLOC;
    for (int s = 0, o = 0; s < 5; s++) { fr[s] = fbuf + o; o += (int)fb[s]; }
    for (int s = 0; s < 5 && rc == PGNO_OK; s++) {
        size_t b = fb[s];
        size_t r = Z.compress(fr[s], b, st[s], sz[s], 1);
        if (Z.iserror(r)) { rc = PGNO_ERR_ZSTD_COMPRESS; break; }
        fsz[s] = r;
    }
    if (rc == PGNO_OK) {
        size_t total = 4 * 8 + fsz[0] + fsz[1] + fsz[2] + fsz[3] + fsz[4];
        if (stream_sizes) {
            for (int s = 0; s < 5; s++) { stream_sizes[s] = sz[s]; stream_sizes[5 + s] = fsz[s]; }
        }
        if (cap < total) {
            rc = PGNO_ERR_DST_TOO_SMALL;
            *out_len = total; /* the "Required size" the reference prints (C5.hpp:423-424) */
        } else {
            uint8_t *p = dst;
            for (int s = 0; s < 5; s++) {
                if (s < 4) { put_u64(p, (uint64_t)fsz[s]); p += 8; }
                memcpy(p, fr[s], fsz[s]);
                p += fsz[s];
            }
            *out_len = total;
        }
    }
    return rc;
}

/* C5 decompress: decompress_signal_N01 (C5.hpp:477-683) behind pgnano::decompress_signal
 * (pgnano.cpp:98-126).  n comes from the caller's destination span (POD5 `samples` column). */
int pgno_c5_decompress(const uint8_t *src, size_t len, int16_t *out, uint32_t n)
{
    if (!zok()) return PGNO_ERR_NO_ZSTD;
    const uint8_t *fp[5];
    uint64_t fl[5];
    unsigned long long cs[5];
    size_t pos = 0;
    for (int s = 0; s < 5; s++) {
        if (s < 4) {
            if (len - pos < 8 || pos > len) return PGNO_ERR_CORRUPT;
            fl[s] = get_u64(src + pos);
            pos += 8;
            if (fl[s] > len - pos) return PGNO_ERR_CORRUPT;
        } else {
            fl[s] = len - pos; /* last frame length is implicit (C5.hpp:560) */
        }
        fp[s] = src + pos;
        cs[s] = Z.fcs(fp[s], (size_t)fl[s]);
        if (Z.iserror((size_t)cs[s])) return PGNO_ERR_NOT_ZSTD;
        pos += (size_t)fl[s];
    }
    uint64_t total = 0;
    for (int s = 0; s < 5; s++) total += cs[s];
    if (total > ((uint64_t)1 << 40)) return PGNO_ERR_ALLOC;
    uint8_t *inter = scratch(0, total ? total : 1);
    if (!inter) return PGNO_ERR_ALLOC;
    uint64_t off = 0, dres[5];
    for (int s = 0; s < 5; s++) {
        size_t r = Z.decompress(inter + off, (size_t)cs[s], fp[s], (size_t)fl[s]);
        if (Z.iserror(r)) return PGNO_ERR_ZSTD_DECOMPRESS;
        dres[s] = r;
        off += cs[s]; /* write_ptr advances by the frame content size (C5.hpp:602,618,635,652) */
    }
    uint64_t consumed = 0;
    int rc = c5_merge(inter, total, dres[1], dres[2], dres[3], out, n, &consumed);
    if (rc != PGNO_OK) return rc;
    if (consumed != total) return PGNO_ERR_REMAINING; /* padding = 0 (pgnano/svb16/decode.hpp:16-21) */
    return PGNO_OK;
}

/* ----------------------------------------------------------------------------------------------
 * VBZ: svb16::encode_scalar<int16_t,true,true> (svb16/encode_scalar.hpp:18-66) then one
 * ZSTD_compress level 1 (signal_compression.cpp:37-78).  keys = 1 bit per sample (ceil(n/8) bytes,
 * svb16.h key_length), data = 1 byte if v < 256 else 2 bytes little endian.
 * -------------------------------------------------------------------------------------------- */
size_t pgno_vbz_bound(uint32_t n)
{
    /* compressed_signal_max_size (signal_compression.cpp:30-35) */
    size_t svb = ((size_t)n >> 3) + ((((size_t)n & 7u) + 7u) >> 3) + 2u * (size_t)n;
    return zok() ? Z.bound(svb) : 0;
}

size_t pgno_vbz_svb_encode(const int16_t *x, uint32_t n, uint8_t *out)
{
    size_t nk = ((size_t)n >> 3) + ((((size_t)n & 7u) + 7u) >> 3);
    if (n == 0) return 0;
    memset(out, 0, nk);
    uint8_t *d = out + nk;
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint16_t cur = (uint16_t)x[i];
        uint16_t v = zz_enc((uint16_t)(cur - prev));
        prev = cur;
        if (v < 256) {
            *d++ = (uint8_t)v;
        } else {
            d[0] = (uint8_t)(v & 0xFF);
            d[1] = (uint8_t)(v >> 8);
            d += 2;
            out[i >> 3] |= (uint8_t)(1u << (i & 7u));
        }
    }
    return (size_t)(d - out);
}

int pgno_vbz_compress(const int16_t *x, uint32_t n, uint8_t *dst, size_t cap, size_t *out_len)
{
    if (!zok()) return PGNO_ERR_NO_ZSTD;
    size_t nk = ((size_t)n >> 3) + ((((size_t)n & 7u) + 7u) >> 3);
    uint8_t *inter = (uint8_t *)malloc(nk + 2 * (size_t)n + 1);
    if (!inter) return PGNO_ERR_ALLOC;
    size_t m = pgno_vbz_svb_encode(x, n, inter);
    size_t r = Z.compress(dst, cap, inter, m, 1);
    free(inter);
    if (Z.iserror(r)) return PGNO_ERR_ZSTD_COMPRESS;
    *out_len = r;
    return PGNO_OK;
}

/* pod5::decompress_signal (signal_compression.cpp:96-141) with svb16::decode_scalar
 * (svb16/decode_scalar.hpp).  The intermediate is the frame content plus svb16's 16 padding bytes
 * (signal_compression.cpp:111-118; decode.hpp:16-23 on x86-64): ZSTD_decompress gets that whole
 * capacity, and "consumed + padding == size" makes any read into the padding the "Remaining data"
 * error.  Reads past the padding are out of bounds in the reference: PGNO_ERR_CORRUPT here.  The
 * SSE path reads the same bytes (it consumes exactly what the scalar decoder consumes). */
#define VBZ_PADDING 16u
int pgno_vbz_decompress(const uint8_t *src, size_t len, int16_t *out, uint32_t n)
{
    if (!zok()) return PGNO_ERR_NO_ZSTD;
    unsigned long long cs = Z.fcs(src, len);
    if (Z.iserror((size_t)cs)) return PGNO_ERR_NOT_ZSTD;
    size_t total = (size_t)cs + VBZ_PADDING;
    uint8_t *inter = (uint8_t *)calloc(total, 1);
    if (!inter) return PGNO_ERR_ALLOC;
    size_t r = Z.decompress(inter, total, src, len);
    if (Z.iserror(r)) { free(inter); return PGNO_ERR_ZSTD_DECOMPRESS; }
    size_t nk = ((size_t)n >> 3) + ((((size_t)n & 7u) + 7u) >> 3);
    if (nk > cs) { free(inter); return nk <= total ? PGNO_ERR_REMAINING : PGNO_ERR_CORRUPT; }
    size_t p = nk;
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        unsigned big = (inter[i >> 3] >> (i & 7u)) & 1u;
        uint16_t v;
        if (!big) {
            if (p >= total) { free(inter); return PGNO_ERR_CORRUPT; }
            v = inter[p++];
        } else {
            if (p + 1 >= total) { free(inter); return PGNO_ERR_CORRUPT; }
            v = (uint16_t)(inter[p] | ((uint16_t)inter[p + 1] << 8));
            p += 2;
        }
        prev = (uint16_t)(zz_dec(v) + prev);
        out[i] = (int16_t)prev;
    }
    free(inter);
    size_t consumed = (n == 0) ? 0 : p;
    if (consumed != cs) return PGNO_ERR_REMAINING;
    return PGNO_OK;
}

/* ----------------------------------------------------------------------------------------------
 * The other compile-time variants of pgnano.cpp:70-92 / 105-125 (utils/compile_all.sh builds one
 * binary per #define COMPRESSOR_*), selected here by a runtime id:
 *   C4   compress_signal_N02   C4.hpp:53-249, 274-470 / 473-679: C5's layout, classes on raw values
 *   C1   compress_signal_KD    C1.hpp:57-194, 202-285 / 289-382: svb16 keys | data, two frames
 *   C2   compress_signal_lh    C2.hpp:52-189, 195-316 / 318-463: keys, every low byte, big high bytes
 *   C3   compress_signal_ll_lh C3.hpp:53-206, 212-354 / 356-503: keys, small low, big low, big high
 *   VBZ0 compress_signal_VBZ1  VBZ_0.hpp:60-307, 316-362 / 364-423: 2-bit keys + nibble data, one
 *        frame compressed straight into the destination span
 * A blob is frames 1..nf-1 each behind a u64 length prefix, then the last frame (implicit length).
 * The pgnano svb16 decoders need no padding (pgnano/svb16/decode.hpp:16-23), so a decode must
 * consume exactly the sum of the frame content sizes.  C1/C2/C3 memcpy into the destination without
 * a capacity check (UB when it is too small); here that is PGNO_ERR_DST_TOO_SMALL with the required
 * size, as C5/C4 report it.
 * -------------------------------------------------------------------------------------------- */
enum { PGNO_V_C5 = 0, PGNO_V_C4 = 1, PGNO_V_C1 = 2, PGNO_V_C2 = 3, PGNO_V_C3 = 4, PGNO_V_VBZ0 = 5 };

static size_t key1_len(uint32_t n) { return ((size_t)n >> 3) + ((((size_t)n & 7u) + 7u) >> 3); } /* svb16_key_length */
static size_t key2_len(uint32_t n) { return ((size_t)n + 3u) / 4u; }                             /* svb16_key_length_2bit */

/* C4 split (encode_scalar_N02, C4.hpp:53-145): v==0 -> 0; v<16 -> nibble v; v<256 -> byte v; else L */
static void c4_split(const int16_t *x, uint32_t n, uint8_t *const st[5], uint64_t sz[5])
{
    for (int i = 0; i < 5; i++) sz[i] = 0;
    if (n == 0) return;
    uint64_t nk = key2_len(n), ns = 0, nm = 0, nl = 0;
    memset(st[0], 0, nk);
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint16_t cur = (uint16_t)x[i];
        uint16_t v = zz_enc((uint16_t)(cur - prev));
        prev = cur;
        unsigned code;
        if (v == 0) {
            code = 0;
        } else if (v < 16) {
            code = 1;
            if ((ns & 1u) == 0) st[1][ns >> 1] = (uint8_t)v;
            else st[1][ns >> 1] |= (uint8_t)(v << 4);
            ns++;
        } else if (v < 256) {
            code = 2;
            st[2][nm++] = (uint8_t)v;
        } else {
            code = 3;
            st[3][nl] = (uint8_t)(v & 0xFFu);
            st[4][nl] = (uint8_t)(v >> 8);
            nl++;
        }
        st[0][i >> 2] |= (uint8_t)(code << (2u * (i & 3u)));
    }
    sz[0] = nk; sz[1] = (ns + 1) / 2; sz[2] = nm; sz[3] = nl; sz[4] = nl;
}

/* C4 merge (decode_scalar_N02, C4.hpp:166-249): C5's walk without the class offsets */
static int c4_merge(const uint8_t *inter, uint64_t total, uint64_t dS, uint64_t dM, uint64_t dLl,
                    int16_t *out, uint32_t n, uint64_t *consumed)
{
    uint64_t kl = key2_len(n);
    uint64_t ps = kl, pm = kl + dS, pl = kl + dS + dM, ph = kl + dS + dM + dLl;
    if (n == 0) { *consumed = ph; return PGNO_OK; }
    uint64_t sn = 0;
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t kb = i >> 2;
        if (kb >= total) return PGNO_ERR_CORRUPT;
        unsigned code = (inter[kb] >> (2u * (i & 3u))) & 3u;
        uint16_t v;
        if (code == 0) {
            v = 0;
        } else if (code == 1) {
            uint64_t b = ps + (sn >> 1);
            if (b >= total) return PGNO_ERR_CORRUPT;
            v = (uint16_t)((sn & 1u) ? (inter[b] >> 4) : (inter[b] & 0xFu));
            sn++;
        } else if (code == 2) {
            if (pm >= total) return PGNO_ERR_CORRUPT;
            v = inter[pm++];
        } else {
            if (pl >= total || ph >= total) return PGNO_ERR_CORRUPT;
            v = (uint16_t)(((unsigned)inter[ph++] << 8) + inter[pl++]);
        }
        prev = (uint16_t)(zz_dec(v) + prev);
        out[i] = (int16_t)prev;
    }
    *consumed = ph;
    return PGNO_OK;
}

/* C2 split (encode_scalar_lh, C2.hpp:52-109): keys 1 bit (v >= 256); low byte of every sample; high
 * byte of the big ones.  C3 split (encode_scalar_ll_lh, C3.hpp:53-110): low byte of small samples;
 * low and high bytes of big ones. */
static void c23_split(const int16_t *x, uint32_t n, uint8_t *const st[5], uint64_t sz[5], int c3)
{
    for (int i = 0; i < 5; i++) sz[i] = 0;
    if (n == 0) return;
    uint64_t nk = key1_len(n), a = 0, b = 0;
    memset(st[0], 0, nk);
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint16_t cur = (uint16_t)x[i];
        uint16_t v = zz_enc((uint16_t)(cur - prev));
        prev = cur;
        int big = v >= 256;
        if (c3) {
            if (big) { st[2][b] = (uint8_t)v; st[3][b] = (uint8_t)(v >> 8); b++; }
            else st[1][a++] = (uint8_t)v;
        } else {
            st[1][a++] = (uint8_t)v;
            if (big) st[2][b++] = (uint8_t)(v >> 8);
        }
        if (big) st[0][i >> 3] |= (uint8_t)(1u << (i & 7u));
    }
    sz[0] = nk; sz[1] = a; sz[2] = b; sz[3] = c3 ? b : 0;
}

/* C2 merge (decode_scalar_lh, C2.hpp:121-189): low bytes from keys_length, high bytes from
 * keys_length + dLow; consumed = one past the last high byte.  C3 merge (decode_scalar_ll_lh,
 * C3.hpp:130-206): small low bytes from keys_length, big low from + dLL, big high from + dLL + dLH. */
static int c23_merge(const uint8_t *inter, uint64_t total, uint64_t d1, uint64_t d2, int16_t *out, uint32_t n,
                     uint64_t *consumed, int c3)
{
    uint64_t kl = key1_len(n);
    if (n == 0) { *consumed = kl; return PGNO_OK; }
    uint64_t pa = kl, pb = kl + d1, ph = c3 ? kl + d1 + d2 : kl + d1;
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t kb = i >> 3;
        if (kb >= total) return PGNO_ERR_CORRUPT;
        int big = (inter[kb] >> (i & 7u)) & 1u;
        uint16_t v;
        if (c3) {
            if (big) {
                if (pb >= total || ph >= total) return PGNO_ERR_CORRUPT;
                v = (uint16_t)(inter[pb++] | ((uint16_t)inter[ph++] << 8));
            } else {
                if (pa >= total) return PGNO_ERR_CORRUPT;
                v = inter[pa++];
            }
        } else {
            if (pa >= total) return PGNO_ERR_CORRUPT;
            v = inter[pa++];
            if (big) {
                if (ph >= total) return PGNO_ERR_CORRUPT;
                v |= (uint16_t)((uint16_t)inter[ph++] << 8);
            }
        }
        prev = (uint16_t)(zz_dec(v) + prev);
        out[i] = (int16_t)prev;
    }
    *consumed = ph;
    return PGNO_OK;
}

/* C1 merge (decode_scalar_KD, C1.hpp:140-179): svb16 data from keys_length, 1 or 2 bytes per sample */
static int c1_merge(const uint8_t *inter, uint64_t total, int16_t *out, uint32_t n, uint64_t *consumed)
{
    uint64_t p = key1_len(n);
    if (n == 0) { *consumed = p; return PGNO_OK; }
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        if ((i >> 3) >= total) return PGNO_ERR_CORRUPT;
        int big = (inter[i >> 3] >> (i & 7u)) & 1u;
        uint16_t v;
        if (!big) {
            if (p >= total) return PGNO_ERR_CORRUPT;
            v = inter[p++];
        } else {
            if (p + 1 >= total) return PGNO_ERR_CORRUPT;
            v = (uint16_t)(inter[p] | ((uint16_t)inter[p + 1] << 8));
            p += 2;
        }
        prev = (uint16_t)(zz_dec(v) + prev);
        out[i] = (int16_t)prev;
    }
    *consumed = p;
    return PGNO_OK;
}

/* VBZ0 encode (encode_scalar_VBZ1, VBZ_0.hpp:60-172): C5's classes and offsets; the value goes to
 * one nibble stream, 1 / 2 / 4 nibbles low first.  Returns keys + data bytes. */
size_t pgno_vbz0_encode(const int16_t *x, uint32_t n, uint8_t *out)
{
    if (n == 0) return 0;
    size_t nk = key2_len(n);
    memset(out, 0, nk);
    uint8_t *d = out + nk;
    uint64_t nib = 0;
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint16_t cur = (uint16_t)x[i];
        uint16_t v = zz_enc((uint16_t)(cur - prev));
        prev = cur;
        unsigned code, cnt;
        if (v == 0) { code = 0; cnt = 0; }
        else if (v <= 16) { code = 1; cnt = 1; v = (uint16_t)(v - 1); }
        else if (v <= 272) { code = 2; cnt = 2; v = (uint16_t)(v - 17); }
        else { code = 3; cnt = 4; v = (uint16_t)(v - 273); }
        for (unsigned k = 0; k < cnt; k++, nib++) {
            unsigned q = (v >> (4 * k)) & 0xFu;
            if ((nib & 1u) == 0) d[nib >> 1] = (uint8_t)q;
            else d[nib >> 1] |= (uint8_t)(q << 4);
        }
        out[i >> 2] |= (uint8_t)(code << (2u * (i & 3u)));
    }
    return nk + (size_t)((nib + 1) / 2);
}

/* VBZ0 decode (decode_scalar_VBZ1, VBZ_0.hpp:185-290) */
static int vbz0_merge(const uint8_t *inter, uint64_t total, int16_t *out, uint32_t n, uint64_t *consumed)
{
    uint64_t kl = key2_len(n), nib = 0;
    if (n == 0) { *consumed = 0; return PGNO_OK; } /* decode_scalar_VBZ1 returns data_span.begin() */
    uint16_t prev = 0;
    for (uint32_t i = 0; i < n; i++) {
        if ((i >> 2) >= total) return PGNO_ERR_CORRUPT;
        unsigned code = (inter[i >> 2] >> (2u * (i & 3u))) & 3u;
        unsigned cnt = code == 0 ? 0 : (code == 1 ? 1 : (code == 2 ? 2 : 4));
        uint16_t v = 0;
        for (unsigned k = 0; k < cnt; k++, nib++) {
            uint64_t b = kl + (nib >> 1);
            if (b >= total) return PGNO_ERR_CORRUPT;
            v |= (uint16_t)(((nib & 1u) ? (inter[b] >> 4) : (inter[b] & 0xFu)) << (4 * k));
        }
        v = (uint16_t)(v + (code == 0 ? 0 : (code == 1 ? 1 : (code == 2 ? 17 : 273))));
        if (code == 0) v = 0;
        prev = (uint16_t)(zz_dec(v) + prev);
        out[i] = (int16_t)prev;
    }
    *consumed = kl + (nib + 1) / 2;
    return PGNO_OK;
}

/* nf frames behind nf-1 u64 length prefixes (the C5 assembly, C5.hpp:409-462, with nf frames) */
static int frames_compress(uint8_t *const st[5], const uint64_t sz[5], int nf, uint8_t *dst, size_t cap,
                           size_t *out_len, uint64_t *stream_sizes)
{
    size_t fb[5], fsz[5] = {0, 0, 0, 0, 0}, ftot = 0;
    for (int s = 0; s < nf; s++) { fb[s] = Z.bound(sz[s]); ftot += fb[s]; }
    uint8_t *fbuf = scratch(1, ftot + 16);
    if (!fbuf) return PGNO_ERR_ALLOC;
    uint8_t *fr[5];
    for (int s = 0, o = 0; s < nf; s++) { fr[s] = fbuf + o; o += (int)fb[s]; }
    for (int s = 0; s < nf; s++) {
        size_t r = Z.compress(fr[s], fb[s], st[s], sz[s], 1);
        if (Z.iserror(r)) return PGNO_ERR_ZSTD_COMPRESS;
        fsz[s] = r;
    }
    size_t total = 8 * (size_t)(nf - 1);
    for (int s = 0; s < nf; s++) total += fsz[s];
    if (stream_sizes) {
        for (int s = 0; s < 5; s++) {
            stream_sizes[s] = s < nf ? sz[s] : 0;
            stream_sizes[5 + s] = s < nf ? fsz[s] : 0;
        }
    }
    *out_len = total;
    if (cap < total) return PGNO_ERR_DST_TOO_SMALL;
    uint8_t *p = dst;
    for (int s = 0; s < nf; s++) {
        if (s < nf - 1) { put_u64(p, (uint64_t)fsz[s]); p += 8; }
        memcpy(p, fr[s], fsz[s]);
        p += fsz[s];
    }
    return PGNO_OK;
}

/* parse + ZSTD_decompress of nf frames into one intermediate (the decompress_signal_* front half) */
static int frames_decompress(const uint8_t *src, size_t len, int nf, uint8_t **inter_out, uint64_t *total_out,
                             uint64_t dres[5])
{
    const uint8_t *fp[5];
    uint64_t fl[5];
    unsigned long long cs[5];
    size_t pos = 0;
    for (int s = 0; s < nf; s++) {
        if (s < nf - 1) {
            if (pos > len || len - pos < 8) return PGNO_ERR_CORRUPT;
            fl[s] = get_u64(src + pos);
            pos += 8;
            if (fl[s] > len - pos) return PGNO_ERR_CORRUPT;
        } else {
            fl[s] = len - pos;
        }
        fp[s] = src + pos;
        cs[s] = Z.fcs(fp[s], (size_t)fl[s]);
        if (Z.iserror((size_t)cs[s])) return PGNO_ERR_NOT_ZSTD;
        pos += (size_t)fl[s];
    }
    uint64_t total = 0;
    for (int s = 0; s < nf; s++) total += cs[s];
    if (total > ((uint64_t)1 << 40)) return PGNO_ERR_ALLOC;
    uint8_t *inter = scratch(0, total ? total : 1);
    if (!inter) return PGNO_ERR_ALLOC;
    uint64_t off = 0;
    for (int s = 0; s < nf; s++) {
        size_t r = Z.decompress(inter + off, (size_t)cs[s], fp[s], (size_t)fl[s]);
        if (Z.iserror(r)) return PGNO_ERR_ZSTD_DECOMPRESS;
        dres[s] = r;
        off += cs[s];
    }
    *inter_out = inter;
    *total_out = total;
    return PGNO_OK;
}

/* stream_sizes (optional, 10 entries): raw stream sizes then frame sizes, as pgno_c5_compress */
int pgno_variant_compress(int variant, const int16_t *x, uint32_t n, uint8_t *dst, size_t cap, size_t *out_len,
                          uint64_t *stream_sizes)
{
    if (!zok()) return PGNO_ERR_NO_ZSTD;
    if (variant == PGNO_V_C5) return pgno_c5_compress(x, n, dst, cap, out_len, stream_sizes);
    size_t need = key2_len(n) + 4 * (size_t)n + 64;
    uint8_t *buf = scratch(0, 2 * need);
    if (!buf) return PGNO_ERR_ALLOC;
    uint8_t *st[5];
    uint64_t sz[5] = {0, 0, 0, 0, 0};
    int nf;
    switch (variant) {
    case PGNO_V_C4:
        st[0] = buf; st[1] = st[0] + key2_len(n) + 1; st[2] = st[1] + n + 1; st[3] = st[2] + n + 1; st[4] = st[3] + n + 1;
        c4_split(x, n, st, sz);
        nf = 5;
        break;
    case PGNO_V_C1: {
        size_t m = pgno_vbz_svb_encode(x, n, buf);
        st[0] = buf; sz[0] = n ? key1_len(n) : 0;
        st[1] = buf + sz[0]; sz[1] = m - sz[0];
        nf = 2;
        break;
    }
    case PGNO_V_C2:
    case PGNO_V_C3:
        st[0] = buf; st[1] = st[0] + key1_len(n) + 1; st[2] = st[1] + n + 1; st[3] = st[2] + n + 1; st[4] = st[3] + n + 1;
        c23_split(x, n, st, sz, variant == PGNO_V_C3);
        nf = variant == PGNO_V_C3 ? 4 : 3;
        break;
    case PGNO_V_VBZ0: {
        size_t m = pgno_vbz0_encode(x, n, buf);
        /* ZSTD_compress straight into the destination span (VBZ_0.hpp:345-350) */
        size_t r = Z.compress(dst, cap, buf, m, 1);
        if (stream_sizes) {
            memset(stream_sizes, 0, 10 * sizeof(uint64_t));
            stream_sizes[0] = m;
            stream_sizes[5] = Z.iserror(r) ? 0 : r;
        }
        if (Z.iserror(r)) return PGNO_ERR_ZSTD_COMPRESS;
        *out_len = r;
        return PGNO_OK;
    }
    default:
        return PGNO_ERR_ALLOC;
    }
    return frames_compress(st, sz, nf, dst, cap, out_len, stream_sizes);
}

int pgno_variant_decompress(int variant, const uint8_t *src, size_t len, int16_t *out, uint32_t n)
{
    if (!zok()) return PGNO_ERR_NO_ZSTD;
    if (variant == PGNO_V_C5) return pgno_c5_decompress(src, len, out, n);
    int nf = variant == PGNO_V_C4 ? 5 : (variant == PGNO_V_C1 ? 2 : (variant == PGNO_V_C2 ? 3 : (variant == PGNO_V_C3 ? 4 : 1)));
    uint8_t *inter = NULL;
    uint64_t total = 0, dres[5] = {0, 0, 0, 0, 0}, consumed = 0;
    int rc = frames_decompress(src, len, nf, &inter, &total, dres);
    if (rc != PGNO_OK) return rc;
    switch (variant) {
    case PGNO_V_C4: rc = c4_merge(inter, total, dres[1], dres[2], dres[3], out, n, &consumed); break;
    case PGNO_V_C1: rc = c1_merge(inter, total, out, n, &consumed); break;
    case PGNO_V_C2: rc = c23_merge(inter, total, dres[1], 0, out, n, &consumed, 0); break;
    case PGNO_V_C3: rc = c23_merge(inter, total, dres[1], dres[2], out, n, &consumed, 1); break;
    case PGNO_V_VBZ0: rc = vbz0_merge(inter, total, out, n, &consumed); break;
    default: return PGNO_ERR_ALLOC;
    }
    if (rc != PGNO_OK) return rc;
    return consumed == total ? PGNO_OK : PGNO_ERR_REMAINING;
}

/* The merge stage alone over a caller-built intermediate (tests/test_oracle_ref.py holds it to the
 * reference's compiled decode_* on the same bytes).  d[s] = decompressed size of frame s, as the
 * reference passes them; *consumed = the count the reference compares with the intermediate size. */
int pgno_variant_merge(int variant, const uint8_t *inter, uint64_t total, const uint64_t d[5], int16_t *out,
                       uint32_t n, uint64_t *consumed)
{
    switch (variant) {
    case PGNO_V_C5: return c5_merge(inter, total, d[1], d[2], d[3], out, n, consumed);
    case PGNO_V_C4: return c4_merge(inter, total, d[1], d[2], d[3], out, n, consumed);
    case PGNO_V_C1: return c1_merge(inter, total, out, n, consumed);
    case PGNO_V_C2: return c23_merge(inter, total, d[1], 0, out, n, consumed, 0);
    case PGNO_V_C3: return c23_merge(inter, total, d[1], d[2], out, n, consumed, 1);
    case PGNO_V_VBZ0: return vbz0_merge(inter, total, out, n, consumed);
    }
    return PGNO_ERR_ALLOC;
}

/* raw streams of a variant (tests: GPU split checks, blobs from other encoder settings) */
int pgno_variant_streams(int variant, const int16_t *x, uint32_t n, uint8_t *out, uint64_t sizes[5])
{
    uint8_t *st[5];
    size_t cap = (size_t)n + 8;
    for (int s = 0; s < 5; s++) { st[s] = out + (size_t)s * 2 * cap; sizes[s] = 0; }
    switch (variant) {
    case PGNO_V_C5: pgno_c5_split(x, n, st[0], st[1], st[2], st[3], st[4], sizes); return 5;
    case PGNO_V_C4: c4_split(x, n, st, sizes); return 5;
    case PGNO_V_C1: {
        size_t m = pgno_vbz_svb_encode(x, n, st[0]);
        sizes[0] = n ? key1_len(n) : 0;
        memmove(st[1], st[0] + sizes[0], m - sizes[0]);
        sizes[1] = m - sizes[0];
        return 2;
    }
    case PGNO_V_C2: c23_split(x, n, st, sizes, 0); return 3;
    case PGNO_V_C3: c23_split(x, n, st, sizes, 1); return 4;
    case PGNO_V_VBZ0: sizes[0] = pgno_vbz0_encode(x, n, st[0]); return 1;
    }
    return 0;
}

/* ----------------------------------------------------------------------------------------------
 * Synthetic nanopore-like reads (SURVEY.md 8d generator; integer-only so the GPU replicates it).
 * Implemented identically in csrc/pgn_synth.h for the device; this copy is the checker's.
 * -------------------------------------------------------------------------------------------- */
static inline uint64_t sm64(uint64_t *s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Counter-based draws so that every sample can be generated independently:
 * draw(r, i, c) = mix64(rb + (8*i + c + 1) * golden), rb = per-read base. */
static inline uint64_t synth_read_base(uint64_t seed, uint64_t r)
{
    return mix64((seed << 32) ^ (r * 0x9E3779B97F4A7C15ull) ^ 0x5851F42D4C957F2Dull);
}
static inline uint64_t synth_draw(uint64_t rb, uint64_t i, unsigned c)
{
    return mix64(rb + (8ull * i + c + 1ull) * 0x9E3779B97F4A7C15ull);
}
/* sum of 12 uniform u16 minus its mean: ~N(0, 65536^2) */
static inline int32_t synth_gauss12(uint64_t a, uint64_t b, uint64_t c)
{
    int32_t s = 0;
    for (int k = 0; k < 4; k++) {
        s += (int32_t)((a >> (16 * k)) & 0xFFFF);
        s += (int32_t)((b >> (16 * k)) & 0xFFFF);
        s += (int32_t)((c >> (16 * k)) & 0xFFFF);
    }
    return s - 393216;
}

/* Piecewise-constant levels (geometric dwell: switch when the top 16 bits of draw c=3 are below
 * p_switch_q16), level ~ N(level_mean, level_sd), additive noise ~ N(0, noise_sd), clamped to
 * int16.  Parameters follow SURVEY.md 8(d): p=0.1 (6554/65536), level 500 +- 60, noise 12. */
void pgno_synth_read(uint64_t seed, uint64_t read_idx, uint32_t n, int16_t *out,
                     uint32_t p_switch_q16, int32_t level_mean, int32_t level_sd, int32_t noise_sd)
{
    uint64_t rb = synth_read_base(seed, read_idx);
    int32_t level = level_mean;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t d3 = synth_draw(rb, i, 3);
        if (i == 0 || (uint32_t)(d3 >> 48) < p_switch_q16) {
            int32_t g = synth_gauss12(synth_draw(rb, i, 4), synth_draw(rb, i, 5), synth_draw(rb, i, 6));
            level = level_mean + (int32_t)(((int64_t)g * level_sd) >> 16);
        }
        int32_t g = synth_gauss12(synth_draw(rb, i, 0), synth_draw(rb, i, 1), synth_draw(rb, i, 2));
        int32_t v = level + (int32_t)(((int64_t)g * noise_sd) >> 16);
        if (v < -32768) v = -32768;
        if (v > 32767) v = 32767;
        out[i] = (int16_t)v;
    }
}
