"""Batched POD5 signal-table transcoding on the GPU.

The reference's ``copy`` tool (src/c++/copy.cpp) rewrites a POD5 file with another signal codec one
chunk at a time through the plugin surface (signal_table_writer.cpp:105-112,
signal_table_reader.cpp:135-139).  Here a whole signal table -- every row is one chunk of at most
102,400 samples (file_writer.cpp:119-143) -- goes through one batched device decode and one batched
device encode (``pgn_*_batch_device``), and the reference's integration check
(test_scripts/double_conversion.py:26-85: ``copy --pgnano`` then ``copy --VBZ`` and compare) is
:func:`double_conversion`.

Tables are pyarrow tables with the POD5 signal-table columns (signal_table_schema.cpp:15-42):
``read_id`` (16-byte uuid), ``signal`` (large_binary: the compressed chunk) and ``samples``
(uint32).  The signal field carries the codec as its extension name, ``minknow.vbz`` or
``pgnano.signal`` (types.cpp), in the field metadata.  :func:`read_pod5_signal_table` extracts the
signal table embedded in a combined POD5 file as a pyarrow table, for callers that work in Arrow.
The file-to-file path needs no Arrow: :mod:`.pod5_file` (include/pgnano_pod5file.h) parses and writes
the combined layout, the footer flatbuffer and the signal table's Arrow IPC file natively, and
``main`` uses it when both paths are ``.pod5`` files.
"""
from __future__ import annotations

import argparse
import json
import sys

import numpy as np

from .codec import PGNanoCodec, VBZCodec

VBZ_EXT = b"minknow.vbz"
PGNANO_EXT = b"pgnano.signal"
_EXT_KEY = b"ARROW:extension:name"


def read_pod5_signal_table(path: str):
    """The signal table of a combined POD5 file: the embedded Arrow IPC file whose schema has
    ``signal`` and ``samples`` columns."""
    import pyarrow as pa
    import pyarrow.ipc as ipc

    raw = open(path, "rb").read()
    pos = 0
    while True:
        start = raw.find(b"ARROW1", pos)
        if start < 0:
            break
        end = raw.find(b"ARROW1", start + 8)
        if end < 0:
            break
        try:
            t = ipc.open_file(pa.BufferReader(raw[start:end + 6])).read_all()
        except pa.ArrowInvalid:
            pos = start + 6
            continue
        if "signal" in t.column_names and "samples" in t.column_names:
            return t
        pos = end + 6
    raise ValueError(f"{path}: no embedded signal table found")


def signal_codec(table) -> str:
    """``vbz`` or ``pgnano`` from the signal field's extension name."""
    md = table.schema.field("signal").metadata or {}
    ext = md.get(_EXT_KEY, VBZ_EXT)
    if ext == VBZ_EXT:
        return "vbz"
    if ext == PGNANO_EXT:
        return "pgnano"
    raise ValueError(f"unknown signal codec {ext!r}")


def _codec(kind: str, device: int, variant: str):
    return VBZCodec(device) if kind == "vbz" else PGNanoCodec(device, variant=variant)


def column_blobs(table):
    """The signal column as (one uint8 buffer, n + 1 offsets into it) without copying per row."""
    col = table.column("signal").combine_chunks()
    validity, off_buf, data_buf = col.buffers()
    offs = np.frombuffer(off_buf, np.int64)[col.offset:col.offset + len(col) + 1].astype(np.int64)
    data = np.frombuffer(data_buf, np.uint8) if data_buf is not None and data_buf.size else np.zeros(1, np.uint8)
    return data[: max(int(offs[-1]), 1)] if len(offs) else data[:1], offs


def decode_signal_column(table, device: int = 0, variant: str = "C5", codec=None):
    """Every chunk of the table decoded in one launch: (samples int16 cuda tensor, sample offsets,
    counts) -- the reader side of the batched path (signal_table_reader.cpp:294-318)."""
    import torch

    data, offs = column_blobs(table)
    counts = np.asarray(table.column("samples").to_numpy(), np.int64)
    n = len(counts)
    dev = torch.device("cuda", device)
    c = codec or _codec(signal_codec(table), device, variant)
    blobs = torch.from_numpy(data.copy()).to(dev)
    bo = torch.from_numpy(offs[:-1].copy()).to(dev)
    bs = torch.from_numpy(np.diff(offs)).to(dev)
    cnt = torch.from_numpy(counts.astype(np.int32)).to(dev)
    samples, so, st = c.decompress_batch(blobs, bo, bs, cnt)
    torch.cuda.synchronize()
    bad = np.nonzero(st.cpu().numpy())[0]
    if bad.size:
        raise RuntimeError(f"decode failed for {bad.size} of {n} chunks (first: row {bad[0]}, "
                           f"status {int(st[bad[0]].item())})")
    return samples, so, cnt


def encode_signal_column(samples, offsets, counts, kind: str, device: int = 0, variant: str = "C5", codec=None):
    """Every chunk encoded in one launch (the writer side, c_api.cpp:1104-1129): a pyarrow
    large_binary array of the blobs, and the per-chunk stream statistics."""
    import pyarrow as pa
    import torch

    c = codec or _codec(kind, device, variant)
    enc = c.compress_batch(samples, offsets, counts, with_stats=True)
    torch.cuda.synchronize()
    st = enc.status.cpu().numpy()
    bad = np.nonzero(st)[0]
    if bad.size:
        raise RuntimeError(f"encode failed for {bad.size} chunks (first: row {bad[0]}, status {int(st[bad[0]])})")
    host = enc.blobs.cpu().numpy()
    bo, bs = enc.offsets.cpu().numpy(), enc.sizes.cpu().numpy()
    # pack the blobs back to back (device blobs sit at capacity-spaced offsets)
    out_offs = np.zeros(len(bs) + 1, np.int64)
    out_offs[1:] = np.cumsum(bs)
    packed = np.empty(int(out_offs[-1]), np.uint8)
    for i in range(len(bs)):
        packed[out_offs[i]:out_offs[i + 1]] = host[bo[i]:bo[i] + bs[i]]
    arr = pa.LargeBinaryArray.from_buffers(pa.large_binary(), len(bs), [None, pa.py_buffer(out_offs),
                                                                       pa.py_buffer(packed)])
    return arr, enc.stats.cpu().numpy()


def transcode_signal_table(table, dst: str = "pgnano", device: int = 0, variant: str = "C5"):
    """The table with its signal column re-encoded (``copy --pgnano`` / ``copy --VBZ``, copy.cpp:36-53):
    one batched decode of every chunk, one batched encode.  Returns (table, stats dict)."""
    import pyarrow as pa
    import pyarrow.compute  # noqa: F401

    samples, so, cnt = decode_signal_column(table, device, variant)
    arr, stats = encode_signal_column(samples, so, cnt, dst, device, variant)
    i = table.schema.get_field_index("signal")
    field = pa.field("signal", pa.large_binary(), metadata={_EXT_KEY: VBZ_EXT if dst == "vbz" else PGNANO_EXT,
                                                            b"ARROW:extension:metadata": b""})
    out = table.set_column(i, field, arr)
    n = int(np.asarray(table.column("samples").to_numpy(), np.int64).sum())
    nbytes = int(pa.compute.sum(pa.compute.binary_length(arr)).as_py() or 0) if len(arr) else 0
    return out, {"chunks": len(arr), "samples": n, "bytes": nbytes, "bits_per_sample": 8.0 * nbytes / max(n, 1),
                 "stream_bytes": stats[:, :5].sum(0).tolist(), "frame_bytes": stats[:, 5:].sum(0).tolist()}


def signals_equal(a, b, device: int = 0, variant: str = "C5") -> bool:
    """ont_check_pod5_files_equal.py:31-71's signal comparison: the decoded signal of every row equal
    (and the same read ids and sample counts)."""
    import torch

    if a.num_rows != b.num_rows:
        return False
    for col in ("read_id", "samples"):
        if col in a.column_names and not a.column(col).equals(b.column(col)):
            return False
    sa, _, _ = decode_signal_column(a, device, variant)
    sb, _, _ = decode_signal_column(b, device, variant)
    return bool(torch.equal(sa, sb))


def double_conversion(table, device: int = 0, variant: str = "C5") -> dict:
    """test_scripts/double_conversion.py:37-69 on a VBZ signal table: VBZ -> pgnano -> VBZ, then the
    signals compared.  Also reports whether the VBZ bytes came back identical (they do: the GPU VBZ
    encoder reproduces the pod5 writer's frames) and both sizes."""
    if signal_codec(table) != "vbz":
        raise ValueError("double_conversion starts from a VBZ table")
    pg, s1 = transcode_signal_table(table, "pgnano", device, variant)
    back, s2 = transcode_signal_table(pg, "vbz", device, variant)
    return {"signals_equal": signals_equal(table, back, device, variant),
            "vbz_bytes_identical": back.column("signal").equals(table.column("signal")),
            "pgnano": s1, "vbz": s2, "pgnano_vs_vbz_ratio": s1["bytes"] / max(s2["bytes"], 1)}


def write_signal_table(table, path: str) -> None:
    import pyarrow.ipc as ipc

    with ipc.new_file(path, table.schema) as w:
        w.write_table(table)


def read_signal_table(path: str):
    import pyarrow as pa
    import pyarrow.ipc as ipc

    with pa.memory_map(path) as f:
        return ipc.open_file(f).read_all()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Transcode the signal table of a POD5 (or Arrow) file on the GPU")
    ap.add_argument("input", help="combined .pod5 file, or an Arrow IPC signal table")
    ap.add_argument("output", nargs="?", help="combined .pod5 file (native writer, other tables copied), or an "
                                              "Arrow IPC file for the transcoded signal table")
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--pgnano", action="store_true", help="write pgnano blobs (default)")
    g.add_argument("--VBZ", action="store_true", help="write VBZ blobs")
    ap.add_argument("--variant", default="C5", help="pgnano variant: C5 (default), C4, C1, C2, C3, VBZ0")
    ap.add_argument("--check", action="store_true", help="run the double conversion on a VBZ input")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    if a.input.endswith(".pod5") and a.output and a.output.endswith(".pod5") and not a.check:
        from .pod5_file import transcode_pod5

        print(json.dumps(transcode_pod5(a.input, a.output, "vbz" if a.VBZ else "pgnano", a.variant, a.device)))
        return 0
    t = read_pod5_signal_table(a.input) if a.input.endswith(".pod5") else read_signal_table(a.input)
    if a.check:
        print(json.dumps(double_conversion(t, a.device, a.variant)))
        return 0
    out, stats = transcode_signal_table(t, "vbz" if a.VBZ else "pgnano", a.device, a.variant)
    if a.output:
        write_signal_table(out, a.output)
    print(json.dumps(stats))
    return 0


if __name__ == "__main__":
    sys.exit(main())
