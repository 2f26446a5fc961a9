"""MI355X-native pgnano (C5) raw nanopore signal codec.

Drop-in for the reference's pgnano plugin surface (pgnano::compress_signal /
pgnano::decompress_signal); the work runs in hand-written gfx950 kernels behind the C ABI in
include/pgnano_hip.h.  See DESIGN.md.
"""
from ._native import NativeLibraryError, PGN_MAX_CHUNK_SAMPLES, load as load_native
from .codec import (
    EncodedBatch,
    PGNanoCodec,
    PGNanoError,
    compress_signal,
    compressed_signal_max_size,
    decompress_signal,
    default_codec,
    pinanoraw_compress_signal,
)

__all__ = [
    "EncodedBatch",
    "NativeLibraryError",
    "PGN_MAX_CHUNK_SAMPLES",
    "PGNanoCodec",
    "PGNanoError",
    "compress_signal",
    "compressed_signal_max_size",
    "decompress_signal",
    "default_codec",
    "load_native",
    "pinanoraw_compress_signal",
]
