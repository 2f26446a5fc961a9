"""ctypes binding of the gfx950 codec library (include/pgnano_hip.h).

The product path has no CPU fallback: if ``_build/libpgnano_hip.so`` is missing or cannot be
loaded, every entry point raises :class:`NativeLibraryError`.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libpgnano_hip.so")
# diagnostic build with per-phase shader-clock timers (tools/phase_profile.py)
PROF_LIB_PATH = os.path.join(_HERE, "_build", "libpgnano_hip_prof.so")

PGN_OK = 0
PGN_ERR_DST_TOO_SMALL = 1
PGN_ERR_NOT_ZSTD = 2
PGN_ERR_ZSTD_DECOMPRESS = 3
PGN_ERR_REMAINING = 4
PGN_ERR_ZSTD_COMPRESS = 5
PGN_ERR_CORRUPT = 6
PGN_ERR_UNSUPPORTED = 9
PGN_ERR_INVALID_ARG = 10
PGN_ERR_HIP = 11
PGN_ERR_NO_DEVICE = 12
PGN_ERR_IO = 13

PGN_POD5_CODEC_VBZ = 100  # include/pgnano_pod5.h
PGN_MAX_CHUNK_SAMPLES = 16777216
# pgn_variant: the reference's compile-time COMPRESSOR_* variants (pgnano.cpp:70-92)
VARIANTS = {"C5": 0, "C4": 1, "C1": 2, "C2": 3, "C3": 4, "VBZ0": 5}
PGN_STATS_PER_CHUNK = 10

# every symbol include/pgnano_hip.h declares: (name, restype, argtypes)
_VP, _SZ, _U64P, _U32P, _I32P = C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p
SIGNATURES = [
    ("pgn_status_string", C.c_char_p, [C.c_int]),
    ("pgn_last_error", C.c_char_p, []),
    ("pgn_ctx_create", C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    ("pgn_ctx_destroy", C.c_int, [_VP]),
    ("pgn_ctx_stream", C.c_void_p, [_VP]),
    ("pgn_compressed_signal_max_size", C.c_size_t, [C.c_size_t]),
    ("pgn_compress_signal", C.c_int, [_VP, _VP, _SZ, _VP, _SZ, C.POINTER(C.c_size_t)]),
    ("pgn_decompress_signal", C.c_int, [_VP, _VP, _SZ, _VP, _SZ]),
    ("pgn_pinanoraw_compress_signal", C.c_int, [_VP, _SZ, _VP, C.POINTER(C.c_size_t)]),
    ("pgn_pod5_vbz_compress_signal", C.c_int, [_VP, _SZ, _VP, C.POINTER(C.c_size_t)]),
    ("pgn_pod5_vbz_decompress_signal", C.c_int, [_VP, _SZ, _SZ, _VP]),
    ("pgn_compress_batch_device", C.c_int,
     [_VP, _SZ, _VP, _U64P, _U32P, _VP, _U64P, _U64P, _U64P, _I32P, _U64P, _VP]),
    ("pgn_decompress_batch_device", C.c_int, [_VP, _SZ, _VP, _U64P, _U64P, _VP, _U64P, _U32P, _I32P, _VP]),
    ("pgn_compress_batch_device_bounded", C.c_int,
     [_VP, C.c_uint32, _SZ, _VP, _U64P, _U32P, _VP, _U64P, _U64P, _U64P, _I32P, _U64P, _VP]),
    ("pgn_decompress_batch_device_bounded", C.c_int,
     [_VP, C.c_uint32, _SZ, _VP, _U64P, _U64P, _VP, _U64P, _U32P, _I32P, _VP]),
    ("pgn_vbz_compressed_signal_max_size", C.c_size_t, [C.c_size_t]),
    ("pgn_vbz_compress_signal", C.c_int, [_VP, _VP, _SZ, _VP, _SZ, C.POINTER(C.c_size_t)]),
    ("pgn_vbz_decompress_signal", C.c_int, [_VP, _VP, _SZ, _VP, _SZ]),
    ("pgn_vbz_compress_batch_device", C.c_int,
     [_VP, _SZ, _VP, _U64P, _U32P, _VP, _U64P, _U64P, _U64P, _I32P, _U64P, _VP]),
    ("pgn_vbz_decompress_batch_device", C.c_int, [_VP, _SZ, _VP, _U64P, _U64P, _VP, _U64P, _U32P, _I32P, _VP]),
    ("pgn_variant_compress_signal", C.c_int, [_VP, C.c_int, _VP, _SZ, _VP, _SZ, C.POINTER(C.c_size_t)]),
    ("pgn_variant_decompress_signal", C.c_int, [_VP, C.c_int, _VP, _SZ, _VP, _SZ]),
    ("pgn_variant_compress_batch_device", C.c_int,
     [_VP, C.c_int, _SZ, _VP, _U64P, _U32P, _VP, _U64P, _U64P, _U64P, _I32P, _U64P, _VP]),
    ("pgn_variant_decompress_batch_device", C.c_int,
     [_VP, C.c_int, _SZ, _VP, _U64P, _U64P, _VP, _U64P, _U32P, _I32P, _VP]),
    ("pgn_synth_reads_device", C.c_int,
     [_VP, _SZ, C.c_uint64, C.c_uint64, C.c_uint64, _VP, _U64P, _U32P, C.c_uint32, C.c_int32, C.c_int32, C.c_int32,
      _VP]),
    ("pgn_debug_phase_cycles", C.c_int, [_VP, _VP, C.c_int]),
    ("pgn_debug_decode_units", C.c_int, [_VP, _VP, C.c_size_t]),
    ("pgn_ctx_kernels", C.c_char_p, [_VP, C.c_int]),
    ("pgn_ctx_last_encode_ms", C.c_float, [_VP]),
    ("pgn_ctx_last_decode_ms", C.c_float, [_VP]),
    # include/pgnano_pod5.h
    ("pgn_pod5_batch_create", C.c_int, [_VP, C.c_int, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("pgn_pod5_batch_destroy", C.c_int, [_VP]),
    ("pgn_pod5_compress_reads", C.c_int, [_VP, C.c_uint32, _VP, _VP, C.POINTER(C.c_size_t), C.POINTER(C.c_void_p),
                                          C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    ("pgn_pod5_decompress_rows", C.c_int, [_VP, C.c_uint32, _VP, _VP, _VP, _VP, _VP]),
    ("pgn_pod5_last_error", C.c_char_p, []),
    # include/pgnano_pod5file.h
    ("pgn_pod5_file_error", C.c_char_p, []),
    ("pgn_pod5_file_open", C.c_int, [C.c_char_p, C.POINTER(C.c_void_p)]),
    ("pgn_pod5_file_close", C.c_int, [_VP]),
    ("pgn_pod5_file_identifier", C.c_char_p, [_VP]),
    ("pgn_pod5_file_software", C.c_char_p, [_VP]),
    ("pgn_pod5_file_pod5_version", C.c_char_p, [_VP]),
    ("pgn_pod5_file_embedded_count", C.c_int, [_VP]),
    ("pgn_pod5_file_embedded", C.c_int, [_VP, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                         C.POINTER(C.c_int)]),
    ("pgn_pod5_signal_info", C.c_int, [_VP, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_int),
                                       C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("pgn_pod5_signal_read", C.c_int, [_VP, _VP, _VP, _VP, _VP]),
    ("pgn_pod5_write_file", C.c_int, [C.c_char_p, _VP, C.c_int, C.c_uint64, _VP, _VP, _VP, _VP, C.c_uint32,
                                      C.c_char_p, _VP]),
    ("pgn_pod5_write_file_reserved", C.c_int, [C.c_char_p, _VP, C.c_int, C.c_uint64, _VP, _VP, _VP, C.c_uint32,
                                               C.c_char_p, _VP, C.c_int, _VP]),
    ("pgn_pod5_signal_batch_row_counts", C.c_int, [_VP, _VP]),
    ("pgn_pod5_write_file_keep_going", C.c_int, [C.c_char_p, _VP, C.c_int, C.c_uint64, _VP, _VP, _VP, _VP, _VP,
                                                 C.c_uint32, _VP, _VP]),
    ("pgn_pod5_transcode_file_ex", C.c_int, [_VP, C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_uint32, C.c_uint32,
                                             _VP, _VP]),
    ("pgn_pod5_transcode_file", C.c_int, [_VP, C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_uint32, _VP]),
    ("pgn_pod5_signal_batch_rows", C.c_int, [_VP, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("pgn_pod5_signal_read_batches", C.c_int, [_VP, _VP, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                               C.POINTER(C.c_uint64), _VP, _VP, _VP, _VP]),
    ("pgn_pod5_transcode_part", C.c_int, [_VP, _VP, _VP, C.c_uint32, C.c_int, C.c_int, C.POINTER(C.c_void_p), _VP]),
    ("pgn_pod5_part_get", C.c_int, [_VP, C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    ("pgn_pod5_part_free", C.c_int, [_VP]),
]


class NativeLibraryError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def load(path: str | None = None) -> C.CDLL:
    """Load (once) and return the codec library; raise if it is not built."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        # PGN_LIB: an alternative build of the same library (A/B measurements of kernel variants)
        p = path or os.environ.get("PGN_LIB") or (PROF_LIB_PATH if os.environ.get("PGN_PHASE_PROFILE") == "1" else LIB_PATH)
        # One HIP runtime per process: PyTorch ships its own libamdhip64 (soname libamdhip64.so.7,
        # but its libraries NEED the unversioned name), so load torch first and let this library
        # bind to the runtime torch already mapped; loading ours first would map a second runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(p):
            raise NativeLibraryError(
                f"{p} is missing: build it with `make -C rawnanoporesignalcompression_amd` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        lib = C.CDLL(p)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib
