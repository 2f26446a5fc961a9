"""ctypes binding of the parity checker (oracle/pgn_oracle.c over libzstd).  Tests only."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libpgn_oracle.so")
MODEL_SO = os.path.join(ROOT, "rawnanoporesignalcompression_amd", "_build", "libpgn_model.so")

OK, DST_TOO_SMALL, NOT_ZSTD, ZSTD_DECOMPRESS, REMAINING, ZSTD_COMPRESS, CORRUPT = 0, 1, 2, 3, 4, 5, 6

_o = None
_m = None


def oracle() -> C.CDLL:
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
        L = C.CDLL(ORACLE_SO)
        L.pgno_zstd_version.restype = C.c_uint
        L.pgno_zstd_path.restype = C.c_char_p
        L.pgno_zstd_load.argtypes = [C.c_char_p]
        L.pgno_zstd_bound.restype = C.c_size_t
        L.pgno_zstd_bound.argtypes = [C.c_size_t]
        L.pgno_zstd_compress1.restype = C.c_size_t
        L.pgno_zstd_compress1.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.pgno_zstd_compress_ex.restype = C.c_size_t
        L.pgno_zstd_compress_ex.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int, C.c_int]
        L.pgno_zstd_decompress.restype = C.c_size_t
        L.pgno_zstd_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.pgno_c5_bound.restype = C.c_size_t
        L.pgno_c5_bound.argtypes = [C.c_uint32]
        L.pgno_c5_compress.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                                       C.c_void_p]
        L.pgno_c5_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32]
        L.pgno_c5_split.argtypes = [C.c_void_p, C.c_uint32] + [C.c_void_p] * 6
        L.pgno_vbz_compress.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        L.pgno_vbz_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32]
        L.pgno_vbz_svb_encode.restype = C.c_size_t
        L.pgno_vbz_svb_encode.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.pgno_vbz_bound.restype = C.c_size_t
        L.pgno_vbz_bound.argtypes = [C.c_uint32]
        L.pgno_variant_compress.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t,
                                            C.POINTER(C.c_size_t), C.c_void_p]
        L.pgno_variant_decompress.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32]
        L.pgno_variant_streams.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
        L.pgno_variant_merge.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.c_void_p]
        L.pgno_vbz0_encode.restype = C.c_size_t
        L.pgno_vbz0_encode.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.pgno_synth_read.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_void_p, C.c_uint32, C.c_int32,
                                      C.c_int32, C.c_int32]
        _o = L
    return _o


def model() -> C.CDLL:
    """Host build of the shared zstd encoder/decoder code (rawnanoporesignalcompression_amd/csrc)."""
    global _m
    if _m is None:
        L = C.CDLL(MODEL_SO)
        L.z1m_compress.restype = C.c_size_t
        L.z1m_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.z1m_decompress.restype = C.c_long
        L.z1m_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.z1m_content_size.restype = C.c_longlong
        L.z1m_content_size.argtypes = [C.c_void_p, C.c_size_t]
        _m = L
    return _m


def _buf(b) -> np.ndarray:
    a = np.frombuffer(bytes(b), dtype=np.uint8)
    return a if a.size else np.zeros(1, np.uint8)


def zstd_compress1(data: bytes | np.ndarray) -> bytes:
    L = oracle()
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data,
                             dtype=np.uint8)
    cap = L.pgno_zstd_bound(a.size)
    out = np.zeros(cap + 16, np.uint8)
    r = L.pgno_zstd_compress1(a.ctypes.data if a.size else 0, a.size, out.ctypes.data, cap)
    assert r != (1 << 64) - 1
    return out[:r].tobytes()


def zstd_compress_ex(data, level: int, window_log: int = 0) -> bytes:
    """libzstd frame at another level / forced window (decoder coverage; the reference writes level 1)."""
    L = oracle()
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data,
                             dtype=np.uint8)
    cap = L.pgno_zstd_bound(a.size) + 64
    out = np.zeros(cap + 16, np.uint8)
    r = L.pgno_zstd_compress_ex(a.ctypes.data if a.size else 0, a.size, out.ctypes.data, cap, level, window_log)
    assert r != (1 << 64) - 1
    return out[:r].tobytes()


def c5_streams(x: np.ndarray) -> list[bytes]:
    """The five raw C5 streams [keys, S, M, Llow, Lhigh] of one chunk (C5.hpp:282-415)."""
    L = oracle()
    x = np.ascontiguousarray(x, dtype=np.int16)
    n = x.size
    bufs = [np.zeros((n + 3) // 4 + 1, np.uint8)] + [np.zeros(n + 1, np.uint8) for _ in range(4)]
    sz = np.zeros(5, np.uint64)
    L.pgno_c5_split(x.ctypes.data if n else 0, n, *[b.ctypes.data for b in bufs], sz.ctypes.data)
    return [bufs[i][: int(sz[i])].tobytes() for i in range(5)]


def c5_assemble(frames: list[bytes]) -> bytes:
    """C5 wire format from five zstd frames: [u64 cK][K][u64 cS][S][u64 cM][M][u64 cLl][Ll][Lh]."""
    out = b""
    for s, f in enumerate(frames):
        if s < 4:
            out += len(f).to_bytes(8, "little")
        out += f
    return out


def c5_compress(x: np.ndarray, cap: int | None = None):
    """Returns (status, blob bytes or required size, stream sizes[10])."""
    L = oracle()
    x = np.ascontiguousarray(x, dtype=np.int16)
    if cap is None:
        cap = L.pgno_c5_bound(x.size)
    out = np.zeros(max(cap, 1), np.uint8)
    ol = C.c_size_t(0)
    st = np.zeros(10, np.uint64)
    rc = L.pgno_c5_compress(x.ctypes.data if x.size else 0, x.size, out.ctypes.data, cap, C.byref(ol), st.ctypes.data)
    if rc == OK:
        return rc, out[: ol.value].tobytes(), st
    return rc, ol.value, st


def c5_decompress(blob: bytes, n: int):
    L = oracle()
    a = _buf(blob)
    out = np.zeros(max(n, 1), np.int16)
    rc = L.pgno_c5_decompress(a.ctypes.data, len(blob), out.ctypes.data, n)
    return rc, out[:n]


def c5_frames_strictly_valid(blob: bytes) -> bool:
    """Every zstd frame of a C5 blob decodes under the strict Huffman end rule (each stream ends exactly
    at its first bit after its symbol count; zstd1_dec.h huf_decode_stream, the rule the GPU decoder
    follows).  libzstd's double-symbol Huffman decoder (HUF_decompress4X2, picked by a speed
    heuristic) also accepts a stream followed by one more short codeword, so a corrupted blob can
    decode under the reference and fail here: tests treat that case as a known divergence."""
    M = model()
    p, frames = 0, []
    for _ in range(4):
        if p + 8 > len(blob):
            return True
        sz = int.from_bytes(blob[p:p + 8], "little")
        if sz > len(blob) - p - 8:
            return True
        frames.append(blob[p + 8:p + 8 + sz])
        p += 8 + sz
    frames.append(blob[p:])
    for f in frames:
        cs = M.z1m_content_size(_buf(f).ctypes.data, len(f))
        cap = max(int(cs), 1) if cs >= 0 else 1 << 20
        out = np.zeros(cap + 64, np.uint8)
        a = _buf(f)
        if M.z1m_decompress(a.ctypes.data, len(f), out.ctypes.data, cap) < 0:
            return False
    return True


def vbz_compress(x: np.ndarray) -> bytes:
    L = oracle()
    x = np.ascontiguousarray(x, dtype=np.int16)
    cap = L.pgno_vbz_bound(x.size)
    out = np.zeros(cap + 16, np.uint8)
    ol = C.c_size_t(0)
    rc = L.pgno_vbz_compress(x.ctypes.data if x.size else 0, x.size, out.ctypes.data, cap, C.byref(ol))
    assert rc == OK, rc
    return out[: ol.value].tobytes()


def vbz_decompress(blob: bytes, n: int):
    L = oracle()
    a = _buf(blob)
    out = np.zeros(max(n, 1), np.int16)
    rc = L.pgno_vbz_decompress(a.ctypes.data, len(blob), out.ctypes.data, n)
    return rc, out[:n]


def synth_read(read_idx: int, n: int, seed: int = 42, p_switch_q16: int = 6554, level_mean: int = 500,
               level_sd: int = 60, noise_sd: int = 12) -> np.ndarray:
    out = np.zeros(max(n, 1), np.int16)
    oracle().pgno_synth_read(seed, read_idx, n, out.ctypes.data, p_switch_q16, level_mean, level_sd, noise_sd)
    return out[:n]


# The compile-time variants of pgnano.cpp:70-92 as runtime ids (same numbering as include/pgnano_hip.h)
VARIANTS = {"C5": 0, "C4": 1, "C1": 2, "C2": 3, "C3": 4, "VBZ0": 5}
VARIANT_FRAMES = {"C5": 5, "C4": 5, "C1": 2, "C2": 3, "C3": 4, "VBZ0": 1}


def variant_compress(variant: str, x: np.ndarray, cap: int | None = None):
    """Returns (status, blob bytes or required size, stream sizes[10])."""
    L = oracle()
    x = np.ascontiguousarray(x, dtype=np.int16)
    if cap is None:
        cap = L.pgno_c5_bound(x.size)  # pgnano::Compressor::compressed_signal_max_size for every variant
    out = np.zeros(max(cap, 1), np.uint8)
    ol = C.c_size_t(0)
    st = np.zeros(10, np.uint64)
    rc = L.pgno_variant_compress(VARIANTS[variant], x.ctypes.data if x.size else 0, x.size, out.ctypes.data, cap,
                                 C.byref(ol), st.ctypes.data)
    if rc == OK:
        return rc, out[: ol.value].tobytes(), st
    return rc, ol.value, st


def variant_decompress(variant: str, blob: bytes, n: int):
    L = oracle()
    a = _buf(blob)
    out = np.zeros(max(n, 1), np.int16)
    rc = L.pgno_variant_decompress(VARIANTS[variant], a.ctypes.data, len(blob), out.ctypes.data, n)
    return rc, out[:n]


def variant_streams(variant: str, x: np.ndarray) -> list[bytes]:
    """The raw streams a variant hands to ZSTD_compress (one per frame)."""
    L = oracle()
    x = np.ascontiguousarray(x, dtype=np.int16)
    cap = x.size + 8
    buf = np.zeros(10 * cap + 64, np.uint8)
    sz = np.zeros(5, np.uint64)
    nf = L.pgno_variant_streams(VARIANTS[variant], x.ctypes.data if x.size else 0, x.size, buf.ctypes.data,
                                sz.ctypes.data)
    return [buf[2 * cap * s: 2 * cap * s + int(sz[s])].tobytes() for s in range(nf)]


def variant_assemble(frames: list[bytes]) -> bytes:
    """nf frames, the first nf-1 behind u64 length prefixes."""
    out = b""
    for s, f in enumerate(frames):
        if s < len(frames) - 1:
            out += len(f).to_bytes(8, "little")
        out += f
    return out


def oracle_variant_merge(variant: str, inter: bytes, d: list[int], n: int):
    """The restatement's merge over an intermediate: (status, samples, consumed count)."""
    L = oracle()
    a = _buf(inter)
    dd = np.zeros(5, np.uint64)
    dd[: len(d)] = d
    out = np.zeros(max(n, 1), np.int16)
    consumed = C.c_uint64(0)
    rc = L.pgno_variant_merge(VARIANTS[variant], a.ctypes.data, len(inter), dd.ctypes.data, out.ctypes.data, n,
                              C.byref(consumed))
    return rc, out[:n], int(consumed.value)


def oracle_vbz_svb_encode(x: np.ndarray) -> bytes:
    x = np.ascontiguousarray(x, dtype=np.int16)
    out = np.zeros(3 * x.size + 16, np.uint8)
    m = oracle().pgno_vbz_svb_encode(x.ctypes.data if x.size else 0, x.size, out.ctypes.data)
    return out[:m].tobytes()


# ------------------------------------------------------------------------------------------------
# The reference's own svb16 stages, compiled verbatim from /root/reference by oracle/ref.mk into
# oracle/_ref/.  They are used only where the reference tree itself is present (this container):
# ref() is None elsewhere, so GPU-box test processes never load them, whether or not the built
# libraries travelled with the tree.
# ------------------------------------------------------------------------------------------------
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libpgn_ref.so")
REF_VBZ_SO = os.path.join(ROOT, "oracle", "_ref", "libpgn_ref_vbz.so")
REF_SRC = "/root/reference/pod5/c++/pod5_format/pgnano/svb16/C5.hpp"
_r = None
_rv = None


def ref_available() -> bool:
    return os.path.exists(REF_SRC)


def ref():
    """libpgn_ref.so (the reference's svb16 split/merge of every variant), built from the reference tree;
    None where the reference sources are absent."""
    global _r, _rv
    if _r is None:
        if not ref_available():
            return None
        if not (os.path.exists(REF_SO) and os.path.exists(REF_VBZ_SO)):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-f", "ref.mk"], check=True,
                           capture_output=True)
        L = C.CDLL(REF_SO)
        L.pgnr_encode.restype = C.c_int
        L.pgnr_encode.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.pgnr_decode.restype = C.c_int64
        L.pgnr_decode.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32]
        L.pgnr_counters.argtypes = [C.c_void_p, C.c_int]
        V = C.CDLL(REF_VBZ_SO)
        V.pgnr_vbz_svb_encode.restype = C.c_size_t
        V.pgnr_vbz_svb_encode.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        V.pgnr_vbz_svb_decode.restype = C.c_size_t
        V.pgnr_vbz_svb_decode.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32]
        V.pgnr_vbz_padding.restype = C.c_size_t
        _r, _rv = L, V
    return _r


def ref_vbz():
    return _rv if ref() is not None else None


def ref_variant_streams(variant: str, x: np.ndarray) -> list[bytes]:
    """The streams the reference's own svb16 encode_* hands to ZSTD_compress, one per frame."""
    L = ref()
    x = np.ascontiguousarray(x, dtype=np.int16)
    n = x.size
    buf = np.zeros(5 * (n + 64) + 3 * n + 64, np.uint8)
    offs = np.zeros(5, np.uint64)
    sz = np.zeros(5, np.uint64)
    nf = L.pgnr_encode(VARIANTS[variant], x.ctypes.data if n else 0, n, buf.ctypes.data, offs.ctypes.data,
                       sz.ctypes.data)
    assert nf > 0
    return [buf[int(offs[s]): int(offs[s]) + int(sz[s])].tobytes() for s in range(nf)]


def ref_counters(reset: bool = True) -> dict:
    """number_small / number_medium / number_large as the reference's encode_scalar_N01 counts them."""
    out = np.zeros(10, np.int64)
    ref().pgnr_counters(out.ctypes.data, 1 if reset else 0)
    return {"small": int(out[0]), "medium": int(out[1]), "large": int(out[2])}


def ref_variant_merge(variant: str, inter: bytes, d: list[int], n: int):
    """The reference's decode_* over an intermediate: (samples, consumed count)."""
    a = _buf(inter)
    dd = np.zeros(5, np.uint64)
    dd[: len(d)] = d
    out = np.zeros(max(n, 1), np.int16)
    consumed = ref().pgnr_decode(VARIANTS[variant], a.ctypes.data, len(inter), dd.ctypes.data, out.ctypes.data, n)
    return out[:n], int(consumed)


def ref_vbz_svb_encode(x: np.ndarray) -> bytes:
    x = np.ascontiguousarray(x, dtype=np.int16)
    out = np.zeros(3 * x.size + 16, np.uint8)
    m = ref_vbz().pgnr_vbz_svb_encode(x.ctypes.data if x.size else 0, x.size, out.ctypes.data)
    return out[:m].tobytes()


def ref_vbz_svb_decode(inter: bytes, n: int):
    """(samples, consumed) from the reference's svb16::decode; the buffer carries its padding bytes."""
    V = ref_vbz()
    pad = int(V.pgnr_vbz_padding())
    a = np.zeros(len(inter) + pad + 16, np.uint8)
    a[: len(inter)] = np.frombuffer(inter, np.uint8)
    out = np.zeros(max(n, 1), np.int16)
    consumed = V.pgnr_vbz_svb_decode(a.ctypes.data, len(inter) + pad, out.ctypes.data, n)
    return out[:n], int(consumed)
