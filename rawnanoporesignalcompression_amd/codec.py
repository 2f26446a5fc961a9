"""Host-side mirror of the reference's pgnano plugin surface, over the C ABI.

Reference interface (tomas-gr/RawNanoporeSignalCompression):

* ``pgnano::compress_signal(samples, pool, read_data, is_last_batch) -> Result<Buffer>``
  (pod5/c++/pod5_format/pgnano/pgnano.h:19-23, pgnano.cpp:59-96): allocates
  ``compressed_signal_max_size`` bytes, runs the compiled variant (C5, C5.hpp:282-474), returns the
  resized buffer or an ``Invalid`` status.
* ``pgnano::decompress_signal(compressed, pool, destination, state) -> Status``
  (pgnano.h:13-17, pgnano.cpp:98-126 -> C5.hpp:477-683).
* ``pod5_pinanoraw_compress_signal`` (c_api.cpp:1217-1253).
* the pod5 baseline codec VBZ, ``pod5::compress_signal`` / ``pod5::decompress_signal`` /
  ``pod5::compressed_signal_max_size`` (pod5/c++/pod5_format/signal_compression.cpp:14-141), as
  :class:`VBZCodec` with the same methods (the ``--VBZ`` side of the reference's copy tool).

``read_data`` / ``is_last_batch`` / ``state`` are accepted and ignored, exactly as C5 ignores them.
Errors raise :class:`PGNanoError` carrying the reference's status message.

The batched device API (:meth:`PGNanoCodec.compress_batch` / :meth:`decompress_batch`) takes
device-resident torch tensors: one launch encodes or decodes every chunk of a batch.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native

MAX_CHUNK_SAMPLES = _native.PGN_MAX_CHUNK_SAMPLES


class PGNanoError(RuntimeError):
    """Mirrors the reference's ``arrow::Status::Invalid`` results."""

    def __init__(self, status: int, detail: str = ""):
        lib = _native.load()
        msg = lib.pgn_status_string(status).decode()
        if status == _native.PGN_ERR_HIP:
            msg += ": " + lib.pgn_last_error().decode()
        if detail:
            msg += f" ({detail})"
        super().__init__(msg)
        self.status = status


def _check(rc: int, detail: str = "") -> None:
    if rc != _native.PGN_OK:
        raise PGNanoError(rc, detail)


def compressed_signal_max_size(sample_count: int) -> int:
    """``pgnano::Compressor::compressed_signal_max_size`` (compressor.h:39-45)."""
    return int(_native.load().pgn_compressed_signal_max_size(sample_count))


def _ptr(t) -> int:
    return t.data_ptr() if t is not None else 0


def _require_device(t, name: str, device: int) -> None:
    """The batch kernels dereference their data pointers on the GPU: a host tensor would fault."""
    if not t.is_cuda or t.device.index != device:
        raise ValueError(f"{name} must be a tensor on cuda:{device} (got {t.device})")


@dataclass
class EncodedBatch:
    blobs: "object"          # torch.uint8 device tensor holding every blob at its offset
    offsets: "object"        # torch.uint64 (as int64) blob offsets
    caps: "object"           # capacities used (compressed_signal_max_size per chunk)
    sizes: "object"          # blob sizes
    status: "object"         # int32 status per chunk
    stats: "object | None"   # (nchunks, 10) raw + frame sizes per stream


class PGNanoCodec:
    """One codec context per HIP device (one process per GPU)."""

    # C-ABI entry points of this codec
    _fn_compress, _fn_decompress = "pgn_compress_signal", "pgn_decompress_signal"
    _fn_compress_batch, _fn_decompress_batch = "pgn_compress_batch_device", "pgn_decompress_batch_device"

    @staticmethod
    def max_size(sample_count: int) -> int:
        return compressed_signal_max_size(sample_count)

    @staticmethod
    def _default_caps(counts):
        import torch

        return torch.clamp(counts.to(torch.int64) * 2 + 26, min=1024)

    def __init__(self, device: int = 0, variant: str = "C5"):
        """variant: the reference's compile-time COMPRESSOR_* choice (pgnano.cpp:70-92) as a runtime
        option -- "C5" (default, the reference default), "C4", "C1", "C2", "C3", "VBZ0"."""
        if variant not in _native.VARIANTS:
            raise ValueError(f"unknown pgnano variant {variant!r}; one of {sorted(_native.VARIANTS)}")
        self.variant = variant
        self._lib = _native.load()
        h = C.c_void_p()
        _check(self._lib.pgn_ctx_create(int(device), C.byref(h)), f"device {device}")
        self._h = h
        self.device = int(device)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.pgn_ctx_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    _VARIANT_FN = {"pgn_compress_signal": "pgn_variant_compress_signal",
                   "pgn_decompress_signal": "pgn_variant_decompress_signal",
                   "pgn_compress_batch_device": "pgn_variant_compress_batch_device",
                   "pgn_decompress_batch_device": "pgn_variant_decompress_batch_device"}

    def _call(self, fn: str, *args):
        """C5 (and VBZ) through their own entry points; the other variants through pgn_variant_*."""
        if getattr(self, "variant", "C5") != "C5" and fn in self._VARIANT_FN:
            return getattr(self._lib, self._VARIANT_FN[fn])(self._h, _native.VARIANTS[self.variant], *args)
        return getattr(self._lib, fn)(self._h, *args)

    def _bounded(self, fn: str, bound: int, *args):
        """The C5 batch calls with a chunk-size bound (pgnano_hip.h *_bounded)."""
        if type(self) is not PGNanoCodec or getattr(self, "variant", "C5") != "C5":
            raise ValueError("max_chunk_samples: the bounded batch calls are C5's")
        return getattr(self._lib, fn)(self._h, bound, *args)

    def _launch_stream(self, stream):
        """The HIP stream a batch call runs on (the caller's, else the context's), made to wait for
        the caller's current stream.  The call's own allocations and fills are issued on it too, so
        they are ordered before the kernels and the caching allocator ties them to that stream.  The
        batch calls end by making the caller's current stream wait for it (an event, no host sync), so
        the outputs are usable there like the results of any torch op."""
        import torch

        s = torch.cuda.ExternalStream(int(stream) if stream else self.stream, device=torch.device("cuda", self.device))
        s.wait_stream(torch.cuda.current_stream())
        return s

    @property
    def stream(self) -> int:
        return int(self._lib.pgn_ctx_stream(self._h) or 0)

    # ---- per-chunk plugin surface (host memory) -------------------------------------------
    def compress_signal(self, samples, read_data=None, is_last_batch: bool = False) -> bytes:
        x = np.ascontiguousarray(samples, dtype=np.int16)
        cap = self.max_size(x.size)
        out = np.empty(cap, dtype=np.uint8)
        size = C.c_size_t(0)
        rc = self._call(self._fn_compress, x.ctypes.data, x.size, out.ctypes.data, cap, C.byref(size))
        if rc == _native.PGN_ERR_DST_TOO_SMALL:
            raise PGNanoError(rc, f"Destination size: {cap}, Required size: {size.value}")
        _check(rc)
        return out[: size.value].tobytes()

    def decompress_signal(self, compressed, destination=None, state=None, sample_count: int | None = None):
        src = np.frombuffer(bytes(compressed), dtype=np.uint8)
        if destination is None:
            if sample_count is None:
                raise ValueError("need a destination array or sample_count")
            destination = np.empty(int(sample_count), dtype=np.int16)
        if destination.dtype != np.int16 or not destination.flags.c_contiguous:
            raise ValueError("destination must be a contiguous int16 array")
        _check(self._call(self._fn_decompress, src.ctypes.data if src.size else 0, src.size, destination.ctypes.data,
                          destination.size))
        return destination

    # ---- batched device API -----------------------------------------------------------------
    def compress_batch(self, samples, sample_offsets, sample_counts, with_stats: bool = False,
                       out=None, out_offsets=None, out_caps=None, stream: int | None = None,
                       max_chunk_samples: int | None = None) -> EncodedBatch:
        """Encode every chunk of a device-resident batch in one launch.

        samples: int16 cuda tensor; sample_offsets: int64 tensor (elements); sample_counts: int32.
        Blobs land at ``out_offsets`` (default: packed with compressed_signal_max_size capacities).
        max_chunk_samples: the caller's bound on the chunk sizes (pgn_compress_batch_device_bounded:
        no host wait when it is at most 262,144).
        """
        import torch

        _require_device(samples, "samples", self.device)
        if out is not None:
            _require_device(out, "out", self.device)
        caller = torch.cuda.current_stream()
        ls = self._launch_stream(stream)
        with torch.cuda.stream(ls):
            dev = samples.device
            n = int(sample_counts.numel())
            counts = sample_counts.to(device=dev, dtype=torch.int32).contiguous()
            offs = sample_offsets.to(device=dev, dtype=torch.int64).contiguous()
            if out_caps is None:
                caps = self._default_caps(counts)
            else:
                caps = out_caps.to(device=dev, dtype=torch.int64).contiguous()
            if out_offsets is None:
                oo = torch.zeros(n, dtype=torch.int64, device=dev)
                if n > 1:
                    oo[1:] = torch.cumsum(caps, 0)[:-1]
            else:
                oo = out_offsets.to(device=dev, dtype=torch.int64).contiguous()
            if out is None:
                total = int((oo[-1] + caps[-1]).item()) if n else 0
                out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
            sizes = torch.zeros(n, dtype=torch.int64, device=dev)
            status = torch.full((n,), -1, dtype=torch.int32, device=dev)
            stats = torch.zeros((n, _native.PGN_STATS_PER_CHUNK), dtype=torch.int64, device=dev) if with_stats else None
            args = (n, _ptr(samples), _ptr(offs), _ptr(counts), _ptr(out), _ptr(oo), _ptr(caps), _ptr(sizes),
                    _ptr(status), _ptr(stats), ls.cuda_stream)
            if max_chunk_samples is not None:
                _check(self._bounded("pgn_compress_batch_device_bounded", int(max_chunk_samples), *args))
            else:
                _check(self._call(self._fn_compress_batch, *args))
        caller.wait_stream(ls)
        return EncodedBatch(out, oo, caps, sizes, status, stats)

    def decompress_batch(self, blobs, blob_offsets, blob_sizes, sample_counts, out=None, out_offsets=None,
                         stream: int | None = None, max_chunk_samples: int | None = None):
        """Decode a device-resident batch; returns (samples int16 tensor, offsets, status).
        max_chunk_samples: as in :meth:`compress_batch` (pgn_decompress_batch_device_bounded)."""
        import torch

        _require_device(blobs, "blobs", self.device)
        if out is not None:
            _require_device(out, "out", self.device)
        caller = torch.cuda.current_stream()
        ls = self._launch_stream(stream)
        with torch.cuda.stream(ls):
            dev = blobs.device
            n = int(sample_counts.numel())
            counts = sample_counts.to(device=dev, dtype=torch.int32).contiguous()
            if out_offsets is None:
                so = torch.zeros(n, dtype=torch.int64, device=dev)
                if n > 1:
                    so[1:] = torch.cumsum(counts.to(torch.int64), 0)[:-1]
            else:
                so = out_offsets.to(device=dev, dtype=torch.int64).contiguous()
            if out is None:
                total = int(counts.to(torch.int64).sum().item())
                out = torch.empty(max(total, 1), dtype=torch.int16, device=dev)
            bo = blob_offsets.to(device=dev, dtype=torch.int64).contiguous()
            bs = blob_sizes.to(device=dev, dtype=torch.int64).contiguous()
            status = torch.full((n,), -1, dtype=torch.int32, device=dev)
            args = (n, _ptr(blobs), _ptr(bo), _ptr(bs), _ptr(out), _ptr(so), _ptr(counts), _ptr(status), ls.cuda_stream)
            if max_chunk_samples is not None:
                _check(self._bounded("pgn_decompress_batch_device_bounded", int(max_chunk_samples), *args))
            else:
                _check(self._call(self._fn_decompress_batch, *args))
        caller.wait_stream(ls)
        return out, so, status

    def synth_reads(self, nreads: int, samples_per_read, seed: int = 42, first_read: int = 0, read_stride: int = 1,
                    p_switch_q16: int = 6554, level_mean: int = 500, level_sd: int = 60, noise_sd: int = 12,
                    out=None):
        """Generate synthetic reads on the device (bench input); returns (samples, offsets, counts)."""
        import torch

        dev = torch.device("cuda", self.device)
        if isinstance(samples_per_read, int):
            counts = torch.full((nreads,), samples_per_read, dtype=torch.int32, device=dev)
        else:
            counts = torch.as_tensor(samples_per_read, dtype=torch.int32, device=dev)
        offs = torch.zeros(nreads, dtype=torch.int64, device=dev)
        if nreads > 1:
            offs[1:] = torch.cumsum(counts.to(torch.int64), 0)[:-1]
        total = int(counts.to(torch.int64).sum().item())
        if out is None:
            out = torch.empty(max(total, 1), dtype=torch.int16, device=dev)
        _check(self._lib.pgn_synth_reads_device(self._h, nreads, seed, first_read, read_stride, _ptr(out), _ptr(offs),
                                                _ptr(counts), p_switch_q16, level_mean, level_sd, noise_sd, 0))
        return out, offs, counts

    def kernels(self, direction: int) -> str:
        """Kernel names of the C5 batch path (0 = encode, 1 = decode)."""
        return self._lib.pgn_ctx_kernels(self._h, int(direction)).decode()

    def last_encode_ms(self) -> float:
        return float(self._lib.pgn_ctx_last_encode_ms(self._h))

    def last_decode_ms(self) -> float:
        return float(self._lib.pgn_ctx_last_decode_ms(self._h))


def vbz_compressed_signal_max_size(sample_count: int) -> int:
    """``pod5::compressed_signal_max_size`` (signal_compression.cpp:14-19)."""
    return int(_native.load().pgn_vbz_compressed_signal_max_size(sample_count))


class VBZCodec(PGNanoCodec):
    """The pod5 VBZ codec (svb16 + zstd level 1) on the GPU: ``pod5::compress_signal`` /
    ``pod5::decompress_signal`` (signal_compression.cpp:21-141), same methods as
    :class:`PGNanoCodec`.  A frame larger than the destination raises "Failed to compress data"."""

    _fn_compress, _fn_decompress = "pgn_vbz_compress_signal", "pgn_vbz_decompress_signal"
    _fn_compress_batch, _fn_decompress_batch = "pgn_vbz_compress_batch_device", "pgn_vbz_decompress_batch_device"

    def __init__(self, device: int = 0):
        super().__init__(device)

    @staticmethod
    def max_size(sample_count: int) -> int:
        return vbz_compressed_signal_max_size(sample_count)

    @staticmethod
    def _default_caps(counts):
        import torch

        c = counts.to(torch.int64)
        svb = (c >> 3) + (((c & 7) + 7) >> 3) + 2 * c
        small = (svb < 128 * 1024).to(torch.int64)
        return svb + (svb >> 8) + small * ((128 * 1024 - svb).clamp(min=0) >> 11)


_default: PGNanoCodec | None = None


def default_codec() -> PGNanoCodec:
    global _default
    if _default is None:
        _default = PGNanoCodec(0)
    return _default


def compress_signal(samples, pool=None, read_data=None, is_last_batch: bool = False) -> bytes:
    """Module-level ``pgnano::compress_signal`` on the default device."""
    return default_codec().compress_signal(samples, read_data, is_last_batch)


def decompress_signal(compressed, pool=None, destination=None, state=None, sample_count: int | None = None):
    """Module-level ``pgnano::decompress_signal`` on the default device."""
    return default_codec().decompress_signal(compressed, destination, state, sample_count)


def pinanoraw_compress_signal(signal, buffer_size: int | None = None) -> bytes:
    """``pod5_pinanoraw_compress_signal`` (c_api.cpp:1217-1253)."""
    lib = _native.load()
    x = np.ascontiguousarray(signal, dtype=np.int16)
    cap = buffer_size if buffer_size is not None else compressed_signal_max_size(x.size)
    out = np.empty(max(cap, 1), dtype=np.uint8)
    size = C.c_size_t(cap)
    _check(lib.pgn_pinanoraw_compress_signal(x.ctypes.data, x.size, out.ctypes.data, C.byref(size)))
    return out[: size.value].tobytes()


def vbz_compress_signal_capi(signal, buffer_size: int | None = None) -> bytes:
    """``pod5_vbz_compress_signal`` (c_api.cpp:1183-1214): the --VBZ codec through the C-API shape."""
    lib = _native.load()
    x = np.ascontiguousarray(signal, dtype=np.int16)
    cap = buffer_size if buffer_size is not None else vbz_compressed_signal_max_size(x.size)
    out = np.empty(max(cap, 1), dtype=np.uint8)
    size = C.c_size_t(cap)
    _check(lib.pgn_pod5_vbz_compress_signal(x.ctypes.data, x.size, out.ctypes.data, C.byref(size)))
    return out[: size.value].tobytes()


def vbz_decompress_signal_capi(compressed, sample_count: int):
    """``pod5_vbz_decompress_signal`` (c_api.cpp:1255-1273)."""
    lib = _native.load()
    src = np.frombuffer(bytes(compressed), dtype=np.uint8)
    out = np.empty(max(int(sample_count), 1), dtype=np.int16)
    _check(lib.pgn_pod5_vbz_decompress_signal(src.ctypes.data if src.size else 0, src.size, int(sample_count),
                                              out.ctypes.data))
    return out[: int(sample_count)]


class Pod5SignalBatch:
    """The batched POD5 signal-table integration (include/pgnano_pod5.h) on a codec's context.

    ``compress_reads(reads)`` is the signal half of ``pod5_add_reads_data`` (c_api.cpp:1104-1129):
    every read is chunked at ``chunk_size`` as the writer does (file_writer.cpp:119-143) and all
    chunks are compressed by one batched launch; it returns the signal column the writer appends
    (``offsets``, ``data``) with the per-chunk ``samples`` and ``read_index``.
    ``decompress_rows(offsets, data, samples)`` decodes a record batch of signal rows
    (signal_table_reader.cpp:294-318) into one int16 array."""

    def __init__(self, codec: PGNanoCodec, chunk_size: int = 0):
        self._codec = codec
        self._lib = codec._lib
        if isinstance(codec, VBZCodec):
            cid = _native.PGN_POD5_CODEC_VBZ
        else:
            cid = _native.VARIANTS[codec.variant]
        h = C.c_void_p()
        _check(self._lib.pgn_pod5_batch_create(codec._h, cid, int(chunk_size), C.byref(h)))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.pgn_pod5_batch_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def compress_reads(self, reads, copy: bool = True):
        """(offsets, data, samples, read_index) of the chunked, compressed reads.  copy=False returns
        views of the batch's own buffers, valid until its next call (as in the C API)."""
        xs = [np.ascontiguousarray(r, dtype=np.int16) for r in reads]
        ptrs = (C.c_void_p * max(len(xs), 1))(*[x.ctypes.data if x.size else None for x in xs])
        sizes = np.array([x.size for x in xs] or [0], dtype=np.uint32)
        n = C.c_size_t(0)
        po, pd, ps, pr = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        rc = self._lib.pgn_pod5_compress_reads(self._h, len(xs), ptrs, sizes.ctypes.data, C.byref(n), C.byref(po),
                                               C.byref(pd), C.byref(ps), C.byref(pr))
        _check(rc, f"chunk {n.value}" if rc else "")
        k = n.value
        cp = (lambda a: a.copy()) if copy else (lambda a: a)
        offsets = cp(np.ctypeslib.as_array((C.c_uint64 * (k + 1)).from_address(po.value)))
        data = (cp(np.ctypeslib.as_array((C.c_uint8 * int(offsets[-1])).from_address(pd.value)))
                if offsets[-1] else np.zeros(0, np.uint8))
        samples = cp(np.ctypeslib.as_array((C.c_uint32 * k).from_address(ps.value))) if k else np.zeros(0, np.uint32)
        read_index = cp(np.ctypeslib.as_array((C.c_uint32 * k).from_address(pr.value))) if k else np.zeros(0, np.uint32)
        return offsets, data, samples, read_index

    def decompress_rows(self, offsets, data, samples, out=None):
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        samples = np.ascontiguousarray(samples, dtype=np.uint32)
        k = samples.size
        # pgn_pod5_decompress_rows reads offsets[k] and the bytes offsets[0] .. offsets[k]
        if offsets.size != k + 1:
            raise ValueError(f"offsets has {offsets.size} entries, expected rows + 1 = {k + 1}")
        if k and (int(offsets[-1]) > data.size or np.any(np.diff(offsets.astype(np.int64)) < 0)):
            raise ValueError("offsets are not monotonic or run past the data buffer")
        total = int(samples.sum())
        if out is None:
            out = np.empty(max(total, 1), dtype=np.int16)
        elif out.dtype != np.int16 or not out.flags.c_contiguous or out.size < total:
            raise ValueError("out must be a contiguous int16 array of at least sum(samples) entries")
        st = np.zeros(max(k, 1), dtype=np.int32)
        _check(self._lib.pgn_pod5_decompress_rows(self._h, k, offsets.ctypes.data, data.ctypes.data if data.size else None,
                                                  samples.ctypes.data, out.ctypes.data, st.ctypes.data))
        return out[:total]
