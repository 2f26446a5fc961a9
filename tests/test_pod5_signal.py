"""Batched POD5 signal-table transcoding (rawnanoporesignalcompression_amd.pod5_signal) on the
reference's own fixture signal table (pod5/test_data/multi_fast5_zip_v3.pod5, committed as
tests/golden/pod5_v3_signal.npz): the copy --pgnano / copy --VBZ double conversion of
test_scripts/double_conversion.py, with one batched launch per direction."""
import hashlib

import numpy as np
import pytest

import _oracle as O
from _golden import golden, real_vbz_chunks


def fixture_table():
    import pyarrow as pa

    chunks = real_vbz_chunks()
    rng = np.random.default_rng(0)
    ids = [rng.bytes(16) for _ in chunks]
    sig = pa.array([b for b, _ in chunks], pa.large_binary())
    field = pa.field("signal", pa.large_binary(), metadata={b"ARROW:extension:name": b"minknow.vbz",
                                                            b"ARROW:extension:metadata": b""})
    return pa.table([pa.array(ids, pa.binary(16)), sig, pa.array([n for _, n in chunks], pa.uint32())],
                    schema=pa.schema([pa.field("read_id", pa.binary(16)), field, pa.field("samples", pa.uint32())]))


def arrow_file_bytes(table) -> bytes:
    import pyarrow as pa
    import pyarrow.ipc as ipc

    sink = pa.BufferOutputStream()
    with ipc.new_file(sink, table.schema) as w:
        w.write_table(table)
    return sink.getvalue().to_pybytes()


def test_signal_table_found_in_combined_layout(tmp_path):
    """A combined POD5 file: signature, section marker, embedded Arrow files (a non-signal table
    first), footer (SPECIFICATION.md "Combined file layout")."""
    import pyarrow as pa

    from rawnanoporesignalcompression_amd.pod5_signal import read_pod5_signal_table, signal_codec

    t = fixture_table()
    other = pa.table({"read_id": pa.array([b"x" * 16], pa.binary(16)), "num_samples": pa.array([5], pa.uint64())})
    marker = bytes(range(16))
    blob = b"\x8bPOD\r\n\x1a\n" + marker + arrow_file_bytes(other) + marker + arrow_file_bytes(t) + marker
    blob += b"footer-flatbuffer" + (17).to_bytes(8, "little") + marker + b"\x8bPOD\r\n\x1a\n"
    p = tmp_path / "f.pod5"
    p.write_bytes(blob)
    got = read_pod5_signal_table(str(p))
    assert got.equals(t) and signal_codec(got) == "vbz"


def test_column_blobs_views_every_row():
    from rawnanoporesignalcompression_amd.pod5_signal import column_blobs

    t = fixture_table()
    for tt in (t, t.slice(3, 7)):
        data, offs = column_blobs(tt)
        rows = tt.column("signal").to_pylist()
        assert len(offs) == len(rows) + 1
        for i, r in enumerate(rows):
            assert data[offs[i]:offs[i + 1]].tobytes() == r


@pytest.mark.gpu
def test_double_conversion_on_reference_fixture():
    """VBZ -> pgnano -> VBZ with one batched launch per direction: the pgnano blobs are the golden C5
    blobs, the signals compare equal, and the VBZ bytes come back identical to the fixture's."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rawnanoporesignalcompression_amd.pod5_signal import double_conversion, transcode_signal_table

    t = fixture_table()
    pg, stats = transcode_signal_table(t, "pgnano")
    for blob, meta in zip(pg.column("signal").to_pylist(), golden()["real"]):
        assert hashlib.sha256(blob).hexdigest() == meta["c5_sha256"], meta["chunk"]
    assert round(stats["bits_per_sample"], 3) == 6.640
    r = double_conversion(t)
    assert r["signals_equal"] and r["vbz_bytes_identical"]
    assert abs(r["pgnano_vs_vbz_ratio"] - 0.9838) < 1e-3  # C5/VBZ = 0.9838 on this fixture
    # another variant through the same path decodes back to the same signal
    c3, _ = transcode_signal_table(t, "pgnano", variant="C3")
    for blob, (vbz, n) in zip(c3.column("signal").to_pylist(), real_vbz_chunks()):
        assert blob == O.variant_compress("C3", O.vbz_decompress(vbz, n)[1])[1]
