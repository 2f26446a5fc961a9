"""MI355X-native pgnano (C5) and VBZ raw nanopore signal codecs.

Drop-in for the reference's pgnano plugin surface (pgnano::compress_signal /
pgnano::decompress_signal); the work runs in hand-written gfx950 kernels behind the C ABI in
include/pgnano_hip.h.  See DESIGN.md.
"""
from ._native import NativeLibraryError, PGN_MAX_CHUNK_SAMPLES, load as load_native
from .codec import (
    EncodedBatch,
    PGNanoCodec,
    PGNanoError,
    Pod5SignalBatch,
    VBZCodec,
    compress_signal,
    compressed_signal_max_size,
    decompress_signal,
    default_codec,
    pinanoraw_compress_signal,
    vbz_compress_signal_capi,
    vbz_compressed_signal_max_size,
    vbz_decompress_signal_capi,
)

__all__ = [
    "EncodedBatch",
    "NativeLibraryError",
    "PGN_MAX_CHUNK_SAMPLES",
    "PGNanoCodec",
    "PGNanoError",
    "Pod5SignalBatch",
    "VBZCodec",
    "compress_signal",
    "compressed_signal_max_size",
    "decompress_signal",
    "default_codec",
    "load_native",
    "pinanoraw_compress_signal",
    "vbz_compress_signal_capi",
    "vbz_compressed_signal_max_size",
    "vbz_decompress_signal_capi",
]
