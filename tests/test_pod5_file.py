"""POD5 container I/O without Arrow (include/pgnano_pod5file.h), CPU only: no compute calls.

Pinned by the reference's own files: the four POD5 fixtures the reference's tests hold
(pod5/test_data/multi_fast5_zip_v{0..3}.pod5; v3 is committed as tests/golden/multi_fast5_zip_v3.pod5)
are parsed by the native reader and compared with pyarrow's reading of the same embedded Arrow
files, and everything the native writer produces is read back by pyarrow (an independent Arrow IPC
implementation) and by an independent pure-Python parse of the footer flatbuffer (footer.fbs)."""
import hashlib
import os
import struct

import numpy as np
import pytest

from _golden import HERE as GOLDEN, golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(GOLDEN, "multi_fast5_zip_v3.pod5")
REF_DATA = "/root/reference/pod5/test_data"
SIG = b"\x8bPOD\r\n\x1a\n"

pa = pytest.importorskip("pyarrow")
ipc = pytest.importorskip("pyarrow.ipc")


def P():
    from rawnanoporesignalcompression_amd import pod5_file

    return pod5_file


def arrow_table(raw: bytes, off: int, ln: int):
    return ipc.open_file(pa.BufferReader(raw[off:off + ln])).read_all()


# ---- an independent flatbuffer reader for the footer (footer.fbs), used to cross-check the native one
def fb_table(b, pos):
    vt = pos - struct.unpack_from("<i", b, pos)[0]
    vsize = struct.unpack_from("<H", b, vt)[0]
    return b, pos, vt, vsize


def fb_field(t, i):
    b, pos, vt, vsize = t
    if 4 + 2 * i + 2 > vsize:
        return None
    o = struct.unpack_from("<H", b, vt + 4 + 2 * i)[0]
    return pos + o if o else None


def fb_str(t, i):
    b = t[0]
    f = fb_field(t, i)
    p = f + struct.unpack_from("<I", b, f)[0]
    n = struct.unpack_from("<I", b, p)[0]
    return b[p + 4:p + 4 + n].decode()


def parse_footer(raw: bytes):
    assert raw[:8] == SIG and raw[-8:] == SIG
    marker = raw[8:24]
    assert raw[-24:-8] == marker
    flen = struct.unpack_from("<q", raw, len(raw) - 32)[0]
    fstart = len(raw) - 32 - flen
    assert raw[fstart - 8:fstart] == b"FOOTER\0\0"
    fb = raw[fstart:fstart + flen]
    root = fb_table(fb, struct.unpack_from("<I", fb, 0)[0])
    f = fb_field(root, 3)
    v = f + struct.unpack_from("<I", fb, f)[0]
    files = []
    for k in range(struct.unpack_from("<I", fb, v)[0]):
        e = v + 4 + 4 * k
        et = fb_table(fb, e + struct.unpack_from("<I", fb, e)[0])
        vals = []
        for i, (fmt, size) in enumerate((("<q", 8), ("<q", 8), ("<h", 2), ("<h", 2))):
            p = fb_field(et, i)
            if p is not None:
                assert p % size == 0, "flatbuffer scalar not aligned to its size (the verifier rejects it)"
            vals.append(struct.unpack_from(fmt, fb, p)[0] if p is not None else 0)
        files.append(tuple(vals))
    return {"identifier": fb_str(root, 0), "software": fb_str(root, 1), "version": fb_str(root, 2),
            "files": files, "marker": marker, "flen": flen}


def fixture_paths():
    paths = [FIXTURE]
    if os.path.isdir(REF_DATA):
        paths += [os.path.join(REF_DATA, f"multi_fast5_zip_v{v}.pod5") for v in range(4)]
    return paths


@pytest.mark.parametrize("path", fixture_paths(), ids=os.path.basename)
def test_reference_fixture_parsed_like_pyarrow(path):
    """Native footer + signal table == the independent footer parse and pyarrow's table."""
    raw = open(path, "rb").read()
    foot = parse_footer(raw)
    with P().Pod5File(path) as f:
        assert f.file_identifier == foot["identifier"]
        assert f.software == foot["software"] and f.pod5_version == foot["version"]
        assert [(o, ln) for _, o, ln in f.embedded] == [(o, ln) for o, ln, _, _ in foot["files"]]
        kinds = {k for k, _, _ in f.embedded}
        assert "signal" in kinds and "reads" in kinds
        t = f.signal_table()
        _, off, ln = next(e for e in f.embedded if e[0] == "signal")
        ref = arrow_table(raw, off, ln)
        assert f.signal_type == "vbz" and f.rows == ref.num_rows == 22
        assert np.array_equal(t.samples, np.asarray(ref.column("samples").to_numpy(), np.uint32))
        assert [bytes(r) for r in ref.column("read_id").to_pylist()] == [bytes(r) for r in t.read_ids]
        blobs = [bytes(b) for b in ref.column("signal").to_pylist()]
        assert all(t.blob(i) == blobs[i] for i in range(len(blobs)))
        assert int(t.samples.sum()) == f.total_samples == 1_548_931


def test_fixture_matches_committed_golden_vectors():
    """The native reader's signal column == the vectors make_golden.py extracted with pyarrow."""
    z = np.load(os.path.join(GOLDEN, "pod5_v3_signal.npz"))
    g = golden()
    with P().Pod5File(FIXTURE) as f:
        t = f.signal_table()
    assert np.array_equal(t.offsets.astype(np.int64), z["vbz_offsets"])
    assert np.array_equal(t.data, z["vbz"]) and np.array_equal(t.samples, z["samples"])
    assert [r.tobytes().hex() for r in t.read_ids] == [c["read_id"] for c in g["real"]]


@pytest.mark.parametrize("rows_per_batch", [1, 5, 22, 100])
def test_write_with_source_reads_back_everywhere(tmp_path, rows_per_batch):
    """copy-shaped write: same signal rows, the source's identifier/metadata, run_info and reads tables
    copied byte for byte; pyarrow reads every embedded table; the footer parses independently."""
    src_raw = open(FIXTURE, "rb").read()
    out = str(tmp_path / "out.pod5")
    marker = bytes(range(16))
    with P().Pod5File(FIXTURE) as src:
        t = src.signal_table()
        P().write_pod5(out, t, source=src, rows_per_batch=rows_per_batch, section_marker=marker)
        raw = open(out, "rb").read()
        foot = parse_footer(raw)
        assert foot["marker"] == marker and foot["identifier"] == src.file_identifier
        assert foot["flen"] % 8 == 0
        assert [f[3] for f in foot["files"]] == [1, 4, 0]  # signal, run_info, reads (file_writer.cpp:300-350)
        for off, ln, fmt, _ in foot["files"]:
            assert off % 8 == 0 and fmt == 0
            pad = (-ln) % 8
            assert raw[off + ln:off + ln + pad] == b"\0" * pad and raw[off + ln + pad:off + ln + pad + 16] == marker
        by_kind = {k: (o, ln) for k, o, ln in src.embedded}
        with P().Pod5File(out) as back:
            assert back.batches == -(-22 // rows_per_batch)
            t2 = back.signal_table()
            for k, o, ln in back.embedded:
                tb = arrow_table(raw, o, ln)
                so, sl = by_kind[k]
                ref = arrow_table(src_raw, so, sl)
                assert tb.num_rows == ref.num_rows and tb.schema.equals(ref.schema, check_metadata=True), k
                if k == "signal":
                    assert tb.equals(ref)
                else:  # (the reads table holds NaNs: compared as bytes)
                    assert raw[o:o + ln] == src_raw[so:so + sl], k
    for a in ("read_ids", "samples", "offsets", "data"):
        assert np.array_equal(getattr(t, a), getattr(t2, a)), a


def test_write_pgnano_and_uncompressed_types(tmp_path):
    """signal_table_schema.cpp:24-33: pgnano.signal over large_binary; large_list<int16> uncompressed."""
    rng = np.random.default_rng(1)
    n = 7
    counts = rng.integers(0, 300, n).astype(np.uint32)
    counts[2] = 0
    ids = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    sig = [rng.integers(-32768, 32767, int(c)).astype(np.int16) for c in counts]
    data = np.frombuffer(b"".join(s.tobytes() for s in sig), np.uint8)
    offs = np.concatenate([[0], np.cumsum(2 * counts.astype(np.uint64))]).astype(np.uint64)
    Pm = P()
    unc = str(tmp_path / "unc.pod5")
    Pm.write_pod5(unc, Pm.SignalTable(ids, counts, offs, data, "uncompressed"), rows_per_batch=3)
    raw = open(unc, "rb").read()
    with Pm.Pod5File(unc) as f:
        assert f.signal_type == "uncompressed" and f.rows == n and f.batches == 3
        assert f.embedded == [("signal", 24, f.embedded[0][2])]
        t = f.signal_table()
        tb = arrow_table(raw, 24, f.embedded[0][2])
        assert str(tb.schema.field("signal").type) == "large_list<item: int16>"
        assert [np.asarray(v, np.int16).tolist() for v in tb.column("signal").to_pylist()] == [s.tolist() for s in sig]
        assert tb.schema.metadata[b"MINKNOW:file_identifier"].decode() == f.file_identifier
        assert f.software == "rawnanoporesignalcompression_amd"
    assert np.array_equal(t.data, data) and np.array_equal(t.offsets, offs)
    # pgnano: opaque blobs
    blobs = [rng.integers(0, 256, int(k)).astype(np.uint8).tobytes() for k in rng.integers(0, 50, n)]
    boffs = np.concatenate([[0], np.cumsum([len(b) for b in blobs])]).astype(np.uint64)
    pg = str(tmp_path / "pg.pod5")
    Pm.write_pod5(pg, Pm.SignalTable(ids, counts, boffs, np.frombuffer(b"".join(blobs), np.uint8), "pgnano"),
                  software="unit test")
    raw = open(pg, "rb").read()
    with Pm.Pod5File(pg) as f:
        assert f.signal_type == "pgnano" and f.software == "unit test"
        t = f.signal_table()
        tb = arrow_table(raw, 24, f.embedded[0][2])
        assert tb.schema.field("signal").metadata[b"ARROW:extension:name"] == b"pgnano.signal"
        assert [bytes(b) for b in tb.column("signal").to_pylist()] == blobs
    assert [t.blob(i) for i in range(n)] == blobs


def test_empty_signal_table(tmp_path):
    Pm = P()
    out = str(tmp_path / "empty.pod5")
    e = np.zeros(0, np.uint8)
    Pm.write_pod5(out, Pm.SignalTable(e.reshape(0, 16), np.zeros(0, np.uint32), np.zeros(1, np.uint64), e, "vbz"))
    raw = open(out, "rb").read()
    with Pm.Pod5File(out) as f:
        assert f.rows == 0 and f.batches == 0 and f.signal_type == "vbz"
        assert arrow_table(raw, 24, f.embedded[0][2]).num_rows == 0


def test_corrupt_and_missing_files_fail_with_status(tmp_path):
    from rawnanoporesignalcompression_amd import _native

    Pm = P()
    with pytest.raises(Pm.Pod5FileError) as e:
        Pm.Pod5File(str(tmp_path / "missing.pod5"))
    assert e.value.status == _native.PGN_ERR_IO
    raw = open(FIXTURE, "rb").read()
    cases = {"truncated": raw[:-1], "no_signature": b"X" + raw[1:], "short": raw[:40],
             "footer_len": raw[:-32] + struct.pack("<q", 1 << 40) + raw[-24:]}
    for name, blob in cases.items():
        p = tmp_path / f"{name}.pod5"
        p.write_bytes(blob)
        with pytest.raises(Pm.Pod5FileError) as e:
            Pm.Pod5File(str(p))
        assert e.value.status == _native.PGN_ERR_CORRUPT, name
    # random corruption of the footer and of the signal table's Arrow metadata never crashes
    rng = np.random.default_rng(7)
    flen = struct.unpack_from("<q", raw, len(raw) - 32)[0]
    regions = [(len(raw) - 32 - flen, len(raw) - 32), (24, 24 + 2048), (1309450 + 24 - 1024, 1309450 + 24)]
    for k in range(300):
        lo, hi = regions[k % 3]
        b = bytearray(raw)
        for _ in range(1 + k % 4):
            b[int(rng.integers(lo, hi))] ^= int(rng.integers(1, 256))
        p = tmp_path / "fuzz.pod5"
        p.write_bytes(bytes(b))
        try:
            with Pm.Pod5File(str(p)) as f:
                f.signal_table()
        except Pm.Pod5FileError as err:
            assert err.status in (_native.PGN_ERR_CORRUPT, _native.PGN_ERR_UNSUPPORTED)


def test_fixture_digest_unchanged():
    """The committed fixture is the reference's multi_fast5_zip_v3.pod5 (same bytes when it is mounted)."""
    h = hashlib.sha256(open(FIXTURE, "rb").read()).hexdigest()
    ref = os.path.join(REF_DATA, "multi_fast5_zip_v3.pod5")
    if os.path.exists(ref):
        assert hashlib.sha256(open(ref, "rb").read()).hexdigest() == h
    assert os.path.getsize(FIXTURE) == 1_323_624


def _signal_arrow_fields(raw: bytes):
    """Byte positions (in the file) of the signal table's first record-batch Block struct, of its
    RecordBatch length and of its Buffer structs, found with the independent flatbuffer reader above
    (Arrow File.fbs: Footer.recordBatches = field 3; Message.header = field 2; RecordBatch: length =
    field 0, buffers = field 2)."""
    foot = parse_footer(raw)
    off, ln = next((o, l) for o, l, _, ctype in foot["files"] if ctype == 1)  # ContentType.SignalTable
    t = raw[off:off + ln]
    flen = struct.unpack_from("<i", t, len(t) - 10)[0]
    fstart = len(t) - 10 - flen
    fb = t[fstart:fstart + flen]
    root = fb_table(fb, struct.unpack_from("<I", fb, 0)[0])
    f = fb_field(root, 3)
    v = f + struct.unpack_from("<I", fb, f)[0]
    block = off + fstart + v + 4  # first Block {int64 offset, int32 metaDataLength, pad, int64 bodyLength}
    boff, mlen = struct.unpack_from("<qi", t, fstart + v + 4)
    m = boff + 8  # continuation marker + length, then the Message flatbuffer
    msg = fb_table(t[m:], struct.unpack_from("<I", t, m)[0])
    h = fb_field(msg, 2)
    rb = fb_table(t[m:], h + struct.unpack_from("<I", t, m + h)[0])
    length = off + m + fb_field(rb, 0)
    bf = fb_field(rb, 2)
    bv = bf + struct.unpack_from("<I", t, m + bf)[0]
    nbuf = struct.unpack_from("<I", t, m + bv)[0]
    buffers = [off + m + bv + 4 + 16 * i for i in range(nbuf)]
    return block, length, buffers


def test_int64_extreme_arrow_fields_fail_with_status(tmp_path):
    """Offsets and lengths near INT64_MAX in the Arrow block, record batch and buffer fields are
    rejected (the checks compare without sums that could wrap)."""
    from rawnanoporesignalcompression_amd import _native

    Pm = P()
    raw = open(FIXTURE, "rb").read()
    block, length, buffers = _signal_arrow_fields(raw)
    assert struct.unpack_from("<q", raw, length)[0] > 0
    big = (1 << 63) - 1
    edits = {
        "block_offset": [(block, "<q", big - 4)],
        "block_body": [(block + 16, "<q", big - 16)],
        "batch_length": [(length, "<q", 1 << 62)],
        "batch_length_wrap": [(length, "<q", (1 << 60) + 1)],
    }
    # the buffers the reader dereferences (the validity bitmaps are empty and never read)
    for i, b in enumerate(b for b in buffers[:8] if struct.unpack_from("<q", raw, b + 8)[0] > 0):
        edits[f"buf{i}_offset"] = [(b, "<q", big - 8)]
        edits[f"buf{i}_length"] = [(b + 8, "<q", big)]
        edits[f"buf{i}_both"] = [(b, "<q", 1 << 62), (b + 8, "<q", 1 << 62)]
    for name, ed in edits.items():
        blob = bytearray(raw)
        for pos, fmt, val in ed:
            struct.pack_into(fmt, blob, pos, val)
        p = tmp_path / f"{name}.pod5"
        p.write_bytes(bytes(blob))
        with pytest.raises(Pm.Pod5FileError) as e:
            with Pm.Pod5File(str(p)) as f:
                f.signal_table()
        assert e.value.status in (_native.PGN_ERR_CORRUPT, _native.PGN_ERR_UNSUPPORTED), name
