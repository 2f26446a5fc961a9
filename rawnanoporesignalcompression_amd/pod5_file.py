"""POD5 container I/O for the signal table without Arrow (include/pgnano_pod5file.h).

The reference reads and writes combined POD5 files through Arrow C++ and flatbuffers
(internal/combined_file_utils.h:85-279, file_writer.cpp:300-350, signal_table_schema.cpp:15-80);
here the native library parses and writes the footer flatbuffer and the signal table's Arrow IPC
file itself, and :func:`transcode_pod5` is ``copy in.pod5 out.pod5 --pgnano | --VBZ`` (src/c++/copy.cpp)
with the signal column decoded and re-encoded by batched GPU launches.

* :class:`Pod5File` -- footer strings, embedded files, and the signal table as numpy arrays
  (read ids, samples, byte offsets, signal bytes);
* :func:`write_pod5` -- a combined file from signal-table rows, copying the other tables of a source;
* :func:`transcode_pod5` -- the GPU transcoder (a HIP device is required; there is no CPU path); with a
  ``torch.distributed`` group of several ranks (one per GPU) the record batches are shared
  round-robin, each rank transcodes its share on its GPU (``pgn_pod5_transcode_part``), the ranks
  exchange only row sizes, rank 0 writes the file's layout and every rank writes its own rows in
  place: one output file, byte-identical to the one-rank output.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native

CONTENT = {0: "reads", 1: "signal", 2: "read_id_index", 3: "other_index", 4: "run_info"}
PGN_ERR_IO = 13  # include/pgnano_hip.h
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

    def row_columns(self) -> tuple[np.ndarray, np.ndarray]:
        """(read ids (rows, 16) uint8, samples (rows,) uint32) without the signal column."""
        ids = np.empty((self.rows, 16), np.uint8)
        samples = np.empty(self.rows, np.uint32)
        rc = self._lib.pgn_pod5_signal_read(self._h, _ptr(ids), _ptr(samples), None, None)
        if rc:
            raise Pod5FileError(rc, f"read {self.path}")
        return ids, samples

    def batch_row_counts(self) -> np.ndarray:
        """Rows of every signal record batch (uint64, one entry per batch)."""
        counts = np.zeros(self.batches, np.uint64)
        if self.batches:
            rc = self._lib.pgn_pod5_signal_batch_row_counts(self._h, counts.ctypes.data)
            if rc:
                raise Pod5FileError(rc, f"batch rows of {self.path}")
        return counts

    def batch_rows(self, batch: int) -> tuple[int, int]:
        """(first row, rows) of signal record batch `batch`."""
        r0, n = C.c_uint64(), C.c_uint64()
        rc = self._lib.pgn_pod5_signal_batch_rows(self._h, int(batch), C.byref(r0), C.byref(n))
        if rc:
            raise Pod5FileError(rc, f"batch {batch} of {self.path}")
        return r0.value, n.value

    def read_batches(self, batch_ids) -> SignalTable:
        """The rows of the given record batches, in that order (offsets relative to the selection)."""
        ids_arr = np.ascontiguousarray(batch_ids, np.uint32)
        rows, nbytes, tot = C.c_uint64(), C.c_uint64(), C.c_uint64()
        rc = self._lib.pgn_pod5_signal_read_batches(self._h, _ptr(ids_arr), ids_arr.size, C.byref(rows),
                                                    C.byref(nbytes), C.byref(tot), None, None, None, None)
        if rc:
            raise Pod5FileError(rc, f"batches {ids_arr.tolist()} of {self.path}")
        n = rows.value
        ids = np.empty((n, 16), np.uint8)
        samples = np.empty(n, np.uint32)
        offs = np.empty(n + 1, np.uint64)
        data = np.empty(nbytes.value, np.uint8)
        rc = self._lib.pgn_pod5_signal_read_batches(self._h, _ptr(ids_arr), ids_arr.size, None, None, None, _ptr(ids),
                                                    _ptr(samples), offs.ctypes.data, _ptr(data))
        if rc:
            raise Pod5FileError(rc, f"batches {ids_arr.tolist()} of {self.path}")
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


class _KeepGoing(C.Structure):  # pgn_pod5_keep_going_result
    _fields_ = [("failed_batches", C.c_uint64), ("dropped_reads", C.c_uint64), ("dropped_rows", C.c_uint64),
                ("orphan_rows", C.c_uint64), ("first_failed_row", C.c_uint64), ("first_status", C.c_int32),
                ("pad", C.c_int32)]

    def as_dict(self) -> dict:
        d = {k: int(getattr(self, k)) for k, _ in self._fields_ if k != "pad"}
        if d["first_failed_row"] == 2**64 - 1:
            d["first_failed_row"] = None
        return d


def write_pod5_keep_going(path: str, table: SignalTable, row_status, source: Pod5File | None = None,
                          rows_per_batch: int = 100, section_marker: bytes | None = None) -> dict:
    """The file the reference's ``copy`` leaves when some rows cannot be written (row_status[i] != 0):
    read batch by read batch of `source`'s reads table, a read's rows up to its first failing one are
    written, that read and the rest of its batch are not (include/pgnano_pod5file.h
    pgn_pod5_write_file_keep_going); returns what was dropped."""
    lib = _native.load()
    ids = np.ascontiguousarray(table.read_ids, np.uint8).reshape(-1, 16)
    samples = np.ascontiguousarray(table.samples, np.uint32)
    offs = np.ascontiguousarray(table.offsets, np.uint64)
    data = np.ascontiguousarray(table.data, np.uint8)
    st = np.ascontiguousarray(row_status, np.int32)
    if offs.size != samples.size + 1 or ids.shape[0] != samples.size or st.size != samples.size:
        raise ValueError("read_ids, samples, offsets and row_status disagree on the row count")
    mk = C.create_string_buffer(bytes(section_marker), 16) if section_marker is not None else None
    res = _KeepGoing()
    rc = lib.pgn_pod5_write_file_keep_going(str(path).encode(), source._h if source is not None else None,
                                            SIGNAL_TYPES[table.signal_type], samples.size, _ptr(ids), _ptr(samples),
                                            offs.ctypes.data, _ptr(data), _ptr(st), int(rows_per_batch),
                                            C.cast(mk, C.c_void_p) if mk else None, C.byref(res))
    if rc:
        raise Pod5FileError(rc, f"write {path}")
    return res.as_dict()


class _TranscodeStats(C.Structure):
    _fields_ = [("rows", C.c_uint64), ("samples", C.c_uint64), ("in_bytes", C.c_uint64), ("out_bytes", C.c_uint64),
                ("decode_ms", C.c_float), ("encode_ms", C.c_float)]


def _stats_dict(rows, samples, in_bytes, out_bytes, decode_ms, encode_ms) -> dict:
    n = max(samples, 1)
    return {"rows": rows, "samples": samples, "in_bytes": in_bytes, "out_bytes": out_bytes,
            "bits_per_sample": 8.0 * out_bytes / n, "decode_ms": decode_ms, "encode_ms": encode_ms}


def transcode_pod5(in_path: str, out_path: str, dst: str = "pgnano", variant: str = "C5", device: int | None = None,
                   rows_per_batch: int = 100, codec=None, group=None, keep_going: bool = False) -> dict:
    """``copy in.pod5 out.pod5 --pgnano`` (dst="pgnano") or ``--VBZ`` (dst="vbz"), or an uncompressed
    signal table (dst="uncompressed"), on the GPU: one batched decode and one batched encode of every
    row, written with the input's read ids, row order, reads and run-info tables.

    With torch.distributed initialised and more than one rank in `group` (default: the world), every
    rank must call this with the same arguments: see :func:`transcode_pod5_ranks`.  `device` defaults
    to 0 (one rank) or LOCAL_RANK (several).

    keep_going: a row the encoder refuses does not fail the call; the file is written as the
    reference's ``copy`` leaves it (:func:`write_pod5_keep_going`), and the result carries
    ``keep_going`` (what was dropped).  One rank only."""
    try:
        import torch.distributed as dist
    except ImportError:  # no torch: one rank (the codec itself needs only the native library)
        dist = None
    if dist is not None and dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if keep_going:
            raise ValueError("keep_going is a single-rank transcode")
        return transcode_pod5_ranks(in_path, out_path, dst, variant, device, rows_per_batch, codec, group)
    from .codec import PGNanoCodec, PGNanoError

    own = codec is None
    c = codec or PGNanoCodec(0 if device is None else device)
    try:
        st = _TranscodeStats()
        kg = _KeepGoing()
        rc = c._lib.pgn_pod5_transcode_file_ex(c._h, str(in_path).encode(), str(out_path).encode(), SIGNAL_TYPES[dst],
                                               _native.VARIANTS[variant], int(rows_per_batch),
                                               1 if keep_going else 0, C.byref(st), C.byref(kg))
        if rc:
            raise PGNanoError(rc, c._lib.pgn_pod5_last_error().decode())
        out = _stats_dict(st.rows, st.samples, st.in_bytes, st.out_bytes, st.decode_ms, st.encode_ms)
        if keep_going:
            out["keep_going"] = kg.as_dict()
        return out
    finally:
        if own:
            c.close()


def _native_part(codec, f: Pod5File, batch_ids, dst: str, variant: str):
    """This rank's share on its GPU: (status, offsets, data, stats)."""
    ids = np.ascontiguousarray(batch_ids, np.uint32)
    st = _TranscodeStats()
    h = C.c_void_p()
    lib = codec._lib
    rc = lib.pgn_pod5_transcode_part(codec._h, f._h, _ptr(ids), ids.size, SIGNAL_TYPES[dst], _native.VARIANTS[variant],
                                     C.byref(h), C.byref(st))
    if rc:
        return rc, lib.pgn_pod5_last_error().decode(errors="replace"), None, None
    try:
        rows, po, pd = C.c_uint64(), C.c_void_p(), C.c_void_p()
        lib.pgn_pod5_part_get(h, C.byref(rows), C.byref(po), C.byref(pd))
        n = rows.value
        offs = np.ctypeslib.as_array(C.cast(po, C.POINTER(C.c_uint64)), (n + 1,)).copy()
        nbytes = int(offs[-1])
        data = (np.ctypeslib.as_array(C.cast(pd, C.POINTER(C.c_uint8)), (nbytes,)).copy() if nbytes
                else np.empty(0, np.uint8))
    finally:
        lib.pgn_pod5_part_free(h)
    return 0, (offs, data), [st.rows, st.samples, st.in_bytes, st.out_bytes], [st.decode_ms, st.encode_ms]


def transcode_pod5_ranks(in_path: str, out_path: str, dst: str = "pgnano", variant: str = "C5",
                         device: int | None = None, rows_per_batch: int = 100, codec=None, group=None,
                         _part=None) -> dict:
    """Multi-GPU ``copy``: one process per GPU, each rank the same call.

    Record batch b of the input's signal table goes to rank b % W (the reference's reader decodes
    whole record batches, signal_table_reader.cpp:294-318; its writer takes whole read batches,
    c_api.cpp:1104-1110), so the ranks share the file with no data exchange.  Each rank transcodes
    its batches with one batched decode and one batched encode on its GPU.  Then the collectives
    carry sizes only (BASELINE north_star: RCCL for the size reduction): an all-gather of (status,
    counts) and one of the rows' compressed sizes.  From them every rank computes the same file
    layout (pgn_pod5_write_file_reserved); rank 0 writes it, with the signal bytes left zero, under a
    temporary name beside out_path (`<out_path>.pgn-tmp-<token>`, the token in the first gather) and
    shares the file's 16-byte section marker; every rank checks the marker at offset 8 of that file
    before it writes its own rows' bytes in place (positioned writes), so no rank writes into a stale
    file of the same name.  Only when every rank has written does rank 0 rename the file to out_path;
    on any failure it is removed and out_path is left as it was.  The file is byte for byte what the
    one-rank call writes.  out_path must be on a filesystem every rank sees.  A failure on any rank --
    also before the first collective (opening the file, creating the codec) -- raises on every rank,
    and no rank waits on a collective another rank never reaches.  Returns the whole job's stats on
    every rank (decode_ms / encode_ms: the slowest rank's).  `_part` replaces the GPU share (tests on
    CPU)."""
    import os

    import torch
    import torch.distributed as dist

    from .codec import PGNanoError

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    root = dist.get_global_rank(group, 0) if group is not None else 0
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", rank))
    nccl = dist.get_backend(group) == "nccl"
    f, own, made, tmp_path = None, False, False, None
    status, msg, counts, times, offs, data = 0, "", [0, 0, 0, 0], [0.0, 0.0], None, None
    try:
        dev = torch.device("cuda", device) if nccl else torch.device("cpu")
        # ---- local phase: anything that fails here becomes this rank's status, so that every rank
        # still reaches the first collective
        try:
            f = Pod5File(in_path)
            mine = list(range(rank, f.batches, world))
            if _part is None:
                from .codec import PGNanoCodec

                if codec is None:
                    codec, own = PGNanoCodec(device), True
                status, payload, c_, t_ = _native_part(codec, f, mine, dst, variant)
            else:
                status, payload, c_, t_ = _part(f, mine, dst, variant)
            if status:
                msg = str(payload)
            else:
                (offs, data), counts, times = payload, c_, t_
        except Exception as e:  # noqa: BLE001 -- reported to every rank below
            status = int(getattr(e, "status", 0) or PGN_ERR_IO)
            msg = f"{type(e).__name__}: {e}"
        # ---- sizes 1: status and counts of every rank (and rank 0's temporary-file token)
        token = int.from_bytes(os.urandom(7), "little") if rank == 0 else 0
        head = torch.tensor([status] + [int(v) for v in counts] + [token], dtype=torch.int64, device=dev)
        heads = [torch.empty_like(head) for _ in range(world)]
        dist.all_gather(heads, head, group=group)
        tm = torch.tensor(times, dtype=torch.float64, device=dev)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX, group=group)
        heads = torch.stack(heads).cpu().numpy()
        tmp_path = f"{out_path}.pgn-tmp-{int(heads[0, -1]):014x}"
        heads = heads[:, :-1]
        bad = [(r, int(heads[r, 0])) for r in range(world) if heads[r, 0]]
        if bad:
            r, s = bad[0]
            raise PGNanoError(s, msg if r == rank else f"rank {r} failed")
        # ---- sizes 2: the compressed size of every row of every rank (padded to the largest part)
        nrow = heads[:, 1].astype(np.int64)
        sz = torch.zeros(int(nrow.max()) if world else 0, dtype=torch.int64, device=dev)
        if nrow[rank]:
            sz[:int(nrow[rank])] = torch.from_numpy(np.diff(offs).astype(np.int64)).to(dev)
        parts = [torch.empty_like(sz) for _ in range(world)]
        dist.all_gather(parts, sz, group=group)
        parts = [p.cpu().numpy() for p in parts]
        # ---- the layout every rank computes the same way: rows back in record-batch order
        sizes, runs = _merge_sizes(f, parts, nrow, world, rank)
        offs_all = np.zeros(f.rows + 1, np.uint64)
        np.cumsum(sizes, out=offs_all[1:])
        ids, samples = f.row_columns()
        pos = np.zeros(f.rows, np.uint64)
        lib = _native.load()
        err = None
        marker = bytes(16)
        if rank == 0:
            made = True
            rc = lib.pgn_pod5_write_file_reserved(tmp_path.encode(), f._h, SIGNAL_TYPES[dst], f.rows, _ptr(ids),
                                                  _ptr(samples), offs_all.ctypes.data, int(rows_per_batch), None,
                                                  None, 1, _ptr(pos))
            if rc:
                err = Pod5FileError(rc, f"write {out_path}")
            else:
                try:
                    marker = _section_marker(tmp_path)
                except OSError as e:
                    err = Pod5FileError(PGN_ERR_IO, f"read back {tmp_path}: {e}")
        else:
            rc = lib.pgn_pod5_write_file_reserved(None, f._h, SIGNAL_TYPES[dst], f.rows, _ptr(ids), _ptr(samples),
                                                  offs_all.ctypes.data, int(rows_per_batch), None, None, 0, _ptr(pos))
            if rc:
                err = Pod5FileError(rc, f"layout of {out_path}")
        # the layout's outcome on every rank, and rank 0's section marker (two int64 words)
        mk = np.frombuffer(marker, np.int64)
        flag = torch.tensor([0 if err is None else 1, int(mk[0]), int(mk[1])], dtype=torch.int64, device=dev)
        flags = [torch.empty_like(flag) for _ in range(world)]
        dist.all_gather(flags, flag, group=group)
        flags = torch.stack(flags).cpu().numpy()
        if err is not None:
            raise err
        if flags[:, 0].any():
            raise Pod5FileError(PGN_ERR_IO, f"another rank failed to lay out {out_path}")
        marker = flags[0, 1:].astype(np.int64).tobytes()
        # ---- every rank writes its own rows in place, then all agree that the file is complete
        try:
            _write_rows_at(tmp_path, pos, sizes, runs, offs, data, marker)
        except OSError as e:
            err = Pod5FileError(PGN_ERR_IO, f"rank {rank}: positioned write to {tmp_path}: {e}")
        flag = torch.tensor([0 if err is None else 1], dtype=torch.int64, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if err is not None:
            raise err
        if int(flag.item()):
            raise Pod5FileError(PGN_ERR_IO, f"another rank failed to write its rows of {out_path}")
        # ---- the complete file takes its name; every rank returns once it has
        if rank == 0:
            try:
                os.replace(tmp_path, out_path)
                made = False
            except OSError as e:
                err = Pod5FileError(PGN_ERR_IO, f"rename {tmp_path} -> {out_path}: {e}")
        flag = torch.tensor([0 if err is None else 1], dtype=torch.int64, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if err is not None:
            raise err
        if int(flag.item()):
            raise Pod5FileError(PGN_ERR_IO, f"rank 0 failed to rename the finished {out_path}")
        tot = heads[:, 1:].sum(axis=0)
        return _stats_dict(int(tot[0]), int(tot[1]), int(tot[2]), int(tot[3]), float(tm[0]), float(tm[1]))
    finally:
        if made:  # rank 0, the file never completed: no partial file stays behind
            try:
                os.unlink(tmp_path)
            except OSError:
                pass
        if own:
            codec.close()
        if f is not None:
            f.close()


def _section_marker(path: str) -> bytes:
    """The 16-byte section marker after the 8-byte signature of a combined POD5 file."""
    with open(path, "rb") as fh:
        fh.seek(8)
        b = fh.read(16)
    if len(b) != 16:
        raise OSError(f"{path}: no section marker")
    return b


def _merge_sizes(f: Pod5File, parts, nrow, world: int, rank: int):
    """Every row's size in record-batch order from the ranks' size lists, and this rank's rows as
    (first row of the table, first row of the part, count) runs."""
    counts = f.batch_row_counts().astype(np.int64)
    first = np.zeros(counts.size + 1, np.int64)
    np.cumsum(counts, out=first[1:])
    sizes = np.zeros(f.rows, np.uint64)
    at = [0] * world
    runs = []
    for b in range(f.batches):
        r, n = b % world, int(counts[b])
        sizes[first[b]:first[b] + n] = parts[r][at[r]:at[r] + n]
        if r == rank and n:
            runs.append((int(first[b]), at[r], n))
        at[r] += n
    if at != [int(v) for v in nrow]:
        raise Pod5FileError(PGN_ERR_IO, "the ranks' parts disagree with the record batches' row counts")
    return sizes, runs


def _write_rows_at(path: str, pos, sizes, runs, offs, data, marker: bytes | None = None) -> None:
    """This rank's rows at their file positions, one write per stretch that is contiguous in the file.
    With `marker`, the file must carry that section marker at offset 8 (the file rank 0 laid out)."""
    import os

    fd = os.open(str(path), os.O_RDWR)
    try:
        if marker is not None and os.pread(fd, 16, 8) != marker:
            raise OSError(f"{path} is not the file laid out for this copy (section marker differs)")
        for row0, p0, n in runs:
            i = 0
            while i < n:
                j = i + 1
                while j < n and int(pos[row0 + j]) == int(pos[row0 + j - 1]) + int(sizes[row0 + j - 1]):
                    j += 1
                lo, hi = int(offs[p0 + i]), int(offs[p0 + j])
                at, buf = int(pos[row0 + i]), memoryview(data[lo:hi])
                while buf.nbytes:
                    w = os.pwrite(fd, buf, at)
                    buf, at = buf[w:], at + w
                i = j
    finally:
        os.close(fd)
