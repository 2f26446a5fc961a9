// ref_vbz.cpp -- TEST INFRASTRUCTURE ONLY.  Compiles the pod5 VBZ codec's own svb16 stage
// (pod5/c++/pod5_format/svb16/encode.hpp, decode.hpp and what they include, used by
// signal_compression.cpp:49-50 and :134-135) straight from /root/reference (include path set by
// oracle/ref.mk) into oracle/_ref/libpgn_ref_vbz.so.  A separate library from libpgn_ref.so because the
// pgnano fork redefines svb16::encode_scalar differently.  Our wrappers; no reference text.
#include <cstddef>
#include <cstdint>

#include <gsl/gsl-lite.hpp>

#include "svb16/decode.hpp"
#include "svb16/encode.hpp"

static uint8_t g_empty[16];

// svb16::encode<int16_t, true, true>(samples, intermediate, n) -> encoded_count (signal_compression.cpp:49)
extern "C" size_t pgnr_vbz_svb_encode(const int16_t *x, uint32_t n, uint8_t *out)
{
    return svb16::encode<int16_t, true, true>(x, out, n);
}

// svb16::decode<int16_t, true, true>(destination, intermediate) -> consumed_count
// (signal_compression.cpp:134-135).  `in` must be readable for total + padding bytes (SSE path).
extern "C" size_t pgnr_vbz_svb_decode(const uint8_t *in, uint64_t total, int16_t *out, uint32_t n)
{
    return svb16::decode<int16_t, true, true>(gsl::make_span(out, (size_t)n),
                                              gsl::make_span(total ? in : g_empty, (size_t)total));
}

// svb16::decode_input_buffer_padding_byte_count() (decode.hpp:16-23)
extern "C" size_t pgnr_vbz_padding(void) { return svb16::decode_input_buffer_padding_byte_count(); }
