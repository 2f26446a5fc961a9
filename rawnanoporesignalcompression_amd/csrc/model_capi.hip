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

long z1m_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap)
{
    DecWork* w = (DecWork*)malloc(sizeof(DecWork));
    long r = decompress_frames(src, n, dst, cap, *w);
    free(w);
    return r;
}

long long z1m_content_size(const uint8_t* src, size_t n)
{
    bool ok = false;
    uint64_t v = frame_content_size(src, n, &ok);
    return ok ? (long long)v : -1;
}

}  // extern "C"
