// ref_prelude.hpp -- TEST INFRASTRUCTURE ONLY (oracle/ref.mk builds oracle/_ref/libpgn_ref.so).
//
// Included ahead of a verbatim fragment of a reference variant header (the extern stat counters
// and the whole `namespace svb16 { ... }` block, extracted by ref.mk with sed and fed to g++ on
// stdin, so no reference source text is ever written into this repository).  Everything included
// here is the reference's own: the pgnano svb16 helpers (common.hpp, svb16.h, encode_scalar.hpp,
// decode_scalar.hpp under pod5/c++/pod5_format/pgnano/svb16/) and the vendored gsl-lite
// (pod5/third_party/include/gsl/gsl-lite.hpp).  No stand-in header is used.
#pragma once
#include <cassert>
#include <cstddef>
#include <cstdint>
#include <cstring>

#include <gsl/gsl-lite.hpp>

#include "common.hpp"
#include "svb16.h"
#include "encode_scalar.hpp"
#include "decode_scalar.hpp"
