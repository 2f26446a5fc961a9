// model_capi.hip -- TEST-ONLY host build of the shared zstd level-1 encoder/decoder code
// (zstd1_model.h / zstd1_dec.h), so the test-suite can fuzz the exact code the GPU kernels run
// against libzstd at host speed.  Never loaded by the product path.
#include <stdlib.h>
#include <string.h>

#include "zstd1_dec.h"
#include "zstd1_model.h"

using namespace pgn::z1;

extern "C" {

// ZSTD_compress(dst, cap, src, n, 1) equivalent; returns size or 0 on error/unsupported.
size_t z1m_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap)
{
    if (n > 0xFFFFFFF0ull || cap < compress_bound(n)) return 0;
    uint32_t* ht = (uint32_t*)calloc((size_t)1 << 15, 4);
    size_t ns = kMaxSrc / 4 + 2;
    Seq* seqs = (Seq*)malloc(ns * sizeof(Seq));
    uint8_t* codes = (uint8_t*)malloc(3 * ns);
    uint8_t* litbuf = (uint8_t*)malloc(kMaxSrc + 1);
    CompressWork* w = (CompressWork*)malloc(sizeof(CompressWork));
    size_t r = compress_serial(dst, src, n, ht, seqs, codes, codes + ns, codes + 2 * ns, litbuf, *w);
    free(w); free(litbuf); free(codes); free(seqs); free(ht);
    return r;
}

// Sequences found by the level-1 match finder (for debugging parity): returns nbSeq.
size_t z1m_sequences(const uint8_t* src, size_t n, uint32_t* out3, size_t maxSeq)
{
    if (n < 7 || n > kMaxSrc) return 0;
    uint32_t* ht = (uint32_t*)calloc((size_t)1 << 15, 4);
    Seq* seqs = (Seq*)malloc((n / 4 + 2) * sizeof(Seq));
    size_t lastLL = 0;
    uint32_t rep[3] = {1, 4, 8};
    size_t nb = fast_search_serial(src, 0, n, level1_params(n), ht, rep, seqs, &lastLL);
    for (size_t i = 0; i < nb && i < maxSeq; i++) {
        out3[3 * i] = seqs[i].litLength; out3[3 * i + 1] = seqs[i].offset; out3[3 * i + 2] = seqs[i].mlBase;
    }
    free(seqs); free(ht);
    return nb;
}

// The encoder's no-match certificate (pgn_zenc.h no_match_certificate), serially: 1 when the
// level-1 search of the single-block frame src[0, n) provably finds no match.
static uint32_t cert_fmix32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}
int z1m_no_match_certificate(const uint8_t* src, size_t n)
{
    if (n < 7 || n > kMaxSrc) return 0;
    const Params p = level1_params(n);
    const long ilimit = (long)n - 8;
    const uint32_t words = 8192 / 8, maxKeys = 2048;  // pgn_zenc.h kCertWords, kCertKeys
    uint64_t* filt = (uint64_t*)calloc(words, 8);
    int ok = 1;
    uint32_t e = 257, k = 0;
    for (;; k++) {
        if (k % 64 == 0 && 2 * (k + 64) > maxKeys) { ok = 0; break; }
        const long pk = (long)e - 256;
        e += e >> 7;
        if (!(pk + 1 < ilimit)) break;
        const uint64_t v8 = rd64(src + pk);
        if (rd32(src + pk + 1) == (uint32_t)(v8 >> 16)) { ok = 0; break; }  // repcode (offset 1) at ip0 + 2
        const uint32_t keys[2] = {(uint32_t)v8 ^ (hash_word(v8, p.hashLog, p.mls) * 0x9E3779B1u),
                                  (uint32_t)(v8 >> 8) ^ (hash_word(v8 >> 8, p.hashLog, p.mls) * 0x9E3779B1u)};
        for (int j = 0; j < 2 && ok; j++) {  // blocked Bloom filter: six bits of one 64-bit word
            const uint32_t a = cert_fmix32(keys[j]), b = cert_fmix32(keys[j] ^ 0x5BD1E995u);
            const uint64_t m = (1ull << (a & 63u)) | (1ull << ((a >> 6) & 63u)) | (1ull << ((a >> 12) & 63u)) |
                               (1ull << ((a >> 18) & 63u)) | (1ull << ((a >> 24) & 63u)) | (1ull << (b & 63u));
            uint64_t* w = filt + ((b >> 6) & (words - 1));
            if ((*w & m) == m) ok = 0;
            *w |= m;
        }
        if (!ok) break;
    }
    free(filt);
    return ok;
}

long z1m_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap)
{
    DecWork* w = (DecWork*)malloc(sizeof(DecWork));
    long r = decompress_frames(src, n, dst, cap, *w);
    free(w);
    return r;
}

// HUF_buildCTable's code lengths for a histogram (maxNbBits 11): decode-table size studies.
unsigned z1m_huf_lengths(const uint32_t* count, unsigned maxSymbolValue, uint8_t* nbBits)
{
    HufNode* nodes = (HufNode*)calloc(1024, sizeof(HufNode));
    huf_sort_serial(nodes + 1, count, maxSymbolValue);
    uint16_t val[256];
    const unsigned r = huf_build_from_sorted(nodes, maxSymbolValue, 11, nbBits, val);
    free(nodes);
    return r;
}

long long z1m_content_size(const uint8_t* src, size_t n)
{
    bool ok = false;
    uint64_t v = frame_content_size(src, n, &ok);
    return ok ? (long long)v : -1;
}

}  // extern "C"
