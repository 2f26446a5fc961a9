"""POD5 container I/O for the signal table without Arrow (include/pgnano_pod5file.h).

The reference reads and writes combined POD5 files through Arrow C++ and flatbuffers
(internal/combined_file_utils.h:85-279, file_writer.cpp:300-350, signal_table_schema.cpp:15-80);
here the native library parses and writes the footer flatbuffer and the signal table's Arrow IPC
file itself, and :func:`transcode_pod5` is ``copy in.pod5 out.pod5 --pgnano | --VBZ`` (src/c++/copy.cpp)
with the signal column decoded and re-encoded by batched GPU launches.

* :class:`Pod5File` -- footer strings, embedded files, and the signal table as numpy arrays
  (read ids, samples, byte offsets, signal bytes);
* :func:`write_pod5` -- a combined file from signal-table rows, copying the other tables of a source;
* :func:`transcode_pod5` -- the GPU transcoder (a HIP device is required; there is no CPU path).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native

CONTENT = {0: "reads", 1: "signal", 2: "read_id_index", 3: "other_index", 4: "run_info"}
SIGNAL_TYPES = {"uncompressed": 0, "vbz": 1, "pgnano": 2}
_SIGNAL_NAMES = {v: k for k, v in SIGNAL_TYPES.items()}


class Pod5FileError(RuntimeError):
    def __init__(self, status: int, what: str):
        lib = _native.load()
        detail = lib.pgn_pod5_file_error().decode(errors="replace")
        super().__init__(f"{what}: {lib.pgn_status_string(status).decode()}: {detail}")
        self.status = status


def _ptr(a) -> int:
    return a.ctypes.data if a is not None and a.size else 0


@dataclass
class SignalTable:
    read_ids: np.ndarray   # (rows, 16) uint8
    samples: np.ndarray    # (rows,) uint32
    offsets: np.ndarray    # (rows + 1,) uint64 byte offsets into data
    data: np.ndarray       # uint8: compressed chunks back to back (int16 bytes when uncompressed)
    signal_type: str       # "vbz" | "pgnano" | "uncompressed"

    @property
    def rows(self) -> int:
        return int(self.samples.size)

    def blob(self, i: int) -> bytes:
        return self.data[self.offsets[i]:self.offsets[i + 1]].tobytes()


class Pod5File:
    """An open combined POD5 file (read into memory and parsed natively)."""

    def __init__(self, path: str):
        self._lib = _native.load()
        h = C.c_void_p()
        rc = self._lib.pgn_pod5_file_open(str(path).encode(), C.byref(h))
        if rc:
            raise Pod5FileError(rc, f"open {path}")
        self._h = h
        self.path = str(path)
        lib = self._lib
        self.file_identifier = lib.pgn_pod5_file_identifier(h).decode(errors="replace")
        self.software = lib.pgn_pod5_file_software(h).decode(errors="replace")
        self.pod5_version = lib.pgn_pod5_file_pod5_version(h).decode(errors="replace")
        self.embedded = []
        for i in range(lib.pgn_pod5_file_embedded_count(h)):
            off, ln, ct = C.c_int64(), C.c_int64(), C.c_int()
            lib.pgn_pod5_file_embedded(h, i, C.byref(off), C.byref(ln), C.byref(ct))
            self.embedded.append((CONTENT.get(ct.value, str(ct.value)), off.value, ln.value))
        rows, nb, st, nbytes, tot = C.c_uint64(), C.c_uint32(), C.c_int(), C.c_uint64(), C.c_uint64()
        lib.pgn_pod5_signal_info(h, C.byref(rows), C.byref(nb), C.byref(st), C.byref(nbytes), C.byref(tot))
        self.rows, self.batches, self.data_bytes, self.total_samples = rows.value, nb.value, nbytes.value, tot.value
        self.signal_type = _SIGNAL_NAMES[st.value]

    def signal_table(self) -> SignalTable:
        n = self.rows
        ids = np.empty((n, 16), np.uint8)
        samples = np.empty(n, np.uint32)
        offs = np.empty(n + 1, np.uint64)
        data = np.empty(self.data_bytes, np.uint8)
        rc = self._lib.pgn_pod5_signal_read(self._h, _ptr(ids), _ptr(samples), offs.ctypes.data, _ptr(data))
        if rc:
            raise Pod5FileError(rc, f"read {self.path}")
        return SignalTable(ids, samples, offs, data, self.signal_type)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.pgn_pod5_file_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def write_pod5(path: str, table: SignalTable, source: Pod5File | None = None, rows_per_batch: int = 100,
               software: str | None = None, section_marker: bytes | None = None) -> None:
    """A combined POD5 file holding `table` as its signal table (record batches of rows_per_batch rows);
    with `source`, its identifier, software, version, schema metadata and other tables are kept."""
    lib = _native.load()
    ids = np.ascontiguousarray(table.read_ids, np.uint8).reshape(-1, 16)
    samples = np.ascontiguousarray(table.samples, np.uint32)
    offs = np.ascontiguousarray(table.offsets, np.uint64)
    data = np.ascontiguousarray(table.data, np.uint8)
    if offs.size != samples.size + 1 or ids.shape[0] != samples.size:
        raise ValueError("read_ids, samples and offsets disagree on the row count")
    if section_marker is not None and len(section_marker) != 16:
        raise ValueError("section_marker must be 16 bytes")
    mk = C.create_string_buffer(bytes(section_marker), 16) if section_marker is not None else None
    rc = lib.pgn_pod5_write_file(str(path).encode(), source._h if source is not None else None,
                                 SIGNAL_TYPES[table.signal_type], samples.size, _ptr(ids), _ptr(samples),
                                 offs.ctypes.data, _ptr(data), int(rows_per_batch),
                                 software.encode() if software else None, C.cast(mk, C.c_void_p) if mk else None)
    if rc:
        raise Pod5FileError(rc, f"write {path}")


class _TranscodeStats(C.Structure):
    _fields_ = [("rows", C.c_uint64), ("samples", C.c_uint64), ("in_bytes", C.c_uint64), ("out_bytes", C.c_uint64),
                ("decode_ms", C.c_float), ("encode_ms", C.c_float)]


def transcode_pod5(in_path: str, out_path: str, dst: str = "pgnano", variant: str = "C5", device: int = 0,
                   rows_per_batch: int = 100, codec=None) -> dict:
    """``copy in.pod5 out.pod5 --pgnano`` (dst="pgnano") or ``--VBZ`` (dst="vbz"), or an uncompressed
    signal table (dst="uncompressed"), on the GPU: one batched decode and one batched encode of every
    row, written with the input's read ids, row order, reads and run-info tables."""
    from .codec import PGNanoCodec, PGNanoError

    own = codec is None
    c = codec or PGNanoCodec(device)
    try:
        st = _TranscodeStats()
        rc = c._lib.pgn_pod5_transcode_file(c._h, str(in_path).encode(), str(out_path).encode(), SIGNAL_TYPES[dst],
                                            _native.VARIANTS[variant], int(rows_per_batch), C.byref(st))
        if rc:
            raise PGNanoError(rc, c._lib.pgn_pod5_last_error().decode())
        n = max(st.samples, 1)
        return {"rows": st.rows, "samples": st.samples, "in_bytes": st.in_bytes, "out_bytes": st.out_bytes,
                "bits_per_sample": 8.0 * st.out_bytes / n, "decode_ms": st.decode_ms, "encode_ms": st.encode_ms}
    finally:
        if own:
            c.close()
