// ref_counters.cpp -- TEST INFRASTRUCTURE ONLY.  Defines the 18 global statistics the reference's
// variant headers declare extern (the reference's own definitions live in its copy tool, copy.cpp:64-85,
// which is not built here) and the variant dispatch of oracle/_ref/libpgn_ref.so.  Our code.
#include <cstdint>

long full_size_keys, full_size_S, full_size_M, full_size_Llow, full_size_Lhigh, full_size_data;
long comp_size_keys, comp_size_S, comp_size_M, comp_size_Llow, comp_size_Lhigh, comp_size_data;
long number_small, number_medium, number_large;
long total_samples;
double compression_time, decompression_time;

#define DECL(v)                                                                                         \
    extern "C" int pgnr_encode_##v(const int16_t *, uint32_t, uint8_t *, uint64_t *, uint64_t *);       \
    extern "C" int64_t pgnr_decode_##v(const uint8_t *, uint64_t, const uint64_t *, int16_t *, uint32_t);
DECL(c5) DECL(c4) DECL(c1) DECL(c2) DECL(c3) DECL(vbz0)
#undef DECL

// variant ids as oracle/pgn_oracle.c (PGNO_V_*) and include/pgnano_hip.h (pgn_variant)
extern "C" int pgnr_encode(int variant, const int16_t *x, uint32_t n, uint8_t *out, uint64_t offs[5],
                           uint64_t sizes[5])
{
    switch (variant) {
    case 0: return pgnr_encode_c5(x, n, out, offs, sizes);
    case 1: return pgnr_encode_c4(x, n, out, offs, sizes);
    case 2: return pgnr_encode_c1(x, n, out, offs, sizes);
    case 3: return pgnr_encode_c2(x, n, out, offs, sizes);
    case 4: return pgnr_encode_c3(x, n, out, offs, sizes);
    case 5: return pgnr_encode_vbz0(x, n, out, offs, sizes);
    }
    return -1;
}

extern "C" int64_t pgnr_decode(int variant, const uint8_t *inter, uint64_t total, const uint64_t d[5], int16_t *out,
                               uint32_t n)
{
    switch (variant) {
    case 0: return pgnr_decode_c5(inter, total, d, out, n);
    case 1: return pgnr_decode_c4(inter, total, d, out, n);
    case 2: return pgnr_decode_c1(inter, total, d, out, n);
    case 3: return pgnr_decode_c2(inter, total, d, out, n);
    case 4: return pgnr_decode_c3(inter, total, d, out, n);
    case 5: return pgnr_decode_vbz0(inter, total, d, out, n);
    }
    return -1;
}

// {number_small, number_medium, number_large, full_size_keys, full_size_S, full_size_M, full_size_Llow,
//  full_size_Lhigh, full_size_data, total_samples}; reset zeroes them.
extern "C" void pgnr_counters(long out[10], int reset)
{
    long *c[10] = {&number_small, &number_medium, &number_large, &full_size_keys, &full_size_S,
                   &full_size_M, &full_size_Llow, &full_size_Lhigh, &full_size_data, &total_samples};
    for (int i = 0; i < 10; i++) {
        if (out) out[i] = *c[i];
        if (reset) *c[i] = 0;
    }
}
