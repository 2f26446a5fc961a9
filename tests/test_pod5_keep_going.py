"""Keep-going copy (pgn_pod5_write_file_keep_going, include/pgnano_pod5file.h), on CPU with given row
statuses: the file the reference's `copy` leaves when rows cannot be written.

Reference semantics: copy walks the reads table batch by batch (src/c++/copy.cpp:139-183) and hands
each read batch to pod5_add_reads_data, which adds reads one at a time and returns at the first
failing one (pod5/c++/pod5_format/c_api.cpp:1118-1127); a read's chunks are added one by one before
its row (file_writer.cpp:86-143), so the chunks before the failing one stay in the signal table; copy
logs the error and goes on with the next batch (copy.cpp:174-176).  Checked with pyarrow on the
reference's fixture, its reads table re-batched three reads per record batch.
"""
import os
import struct

import numpy as np
import pytest

from _golden import HERE as GOLDEN

pa = pytest.importorskip("pyarrow")
ipc = pytest.importorskip("pyarrow.ipc")

from rawnanoporesignalcompression_amd import pod5_file as P  # noqa: E402

FIXTURE = os.path.join(GOLDEN, "multi_fast5_zip_v3.pod5")


def _tables(path):
    raw = open(path, "rb").read()
    with P.Pod5File(path) as f:
        emb = {n: (o, ln) for n, o, ln in f.embedded}
    out = {}
    for name, (o, ln) in emb.items():
        out[name] = ipc.open_file(pa.BufferReader(raw[o:o + ln])).read_all()
    return out


def _fb_table(b, pos):
    vt = pos - struct.unpack_from("<i", b, pos)[0]
    return pos, vt, struct.unpack_from("<H", b, vt)[0]


def _fb_field(b, tab, i):
    pos, vt, vtsize = tab
    if 4 + 2 * i + 2 > vtsize:
        return 0
    o = struct.unpack_from("<H", b, vt + 4 + 2 * i)[0]
    return pos + o if o else 0


def _rebatched(tmp_path, per_batch=3):
    """The fixture with its reads table written back in record batches of `per_batch` reads (pyarrow),
    the footer's length of that table patched (the reads table is the file's last table)."""
    raw = bytearray(open(FIXTURE, "rb").read())
    with P.Pod5File(FIXTURE) as f:
        emb = list(f.embedded)
    name, off, ln = emb[-1]
    assert name == "reads"
    t = ipc.open_file(pa.BufferReader(bytes(raw[off:off + ln]))).read_all()
    sink = pa.BufferOutputStream()
    with ipc.new_file(sink, t.schema) as w:
        for b in t.to_batches(max_chunksize=per_batch):
            w.write_batch(b)
    new = sink.getvalue().to_pybytes()
    end = off + ln
    pad = (-end) % 8
    marker = bytes(raw[end + pad:end + pad + 16])
    tail = bytearray(raw[end + pad + 16:])  # "FOOTER\0\0" + footer flatbuffer + length + marker + signature
    assert tail[:6] == b"FOOTER"
    fb = tail[8:]
    root = _fb_table(fb, struct.unpack_from("<I", fb, 0)[0])
    vec = _fb_field(fb, root, 3)
    vpos = vec + struct.unpack_from("<I", fb, vec)[0]
    for i in range(struct.unpack_from("<I", fb, vpos)[0]):
        ep = vpos + 4 + 4 * i
        tab = _fb_table(fb, ep + struct.unpack_from("<I", fb, ep)[0])
        o = struct.unpack_from("<q", fb, _fb_field(fb, tab, 0))[0]
        if o == off:
            struct.pack_into("<q", fb, _fb_field(fb, tab, 1), len(new))
    tail[8:] = fb
    out = bytes(raw[:off]) + new + bytes((-(off + len(new))) % 8) + marker + bytes(tail)
    p = str(tmp_path / "rebatched.pod5")
    open(p, "wb").write(out)
    return p


def _reads_rows(src):
    """each read's signal rows, and the read batches (lists of read indices)"""
    raw = open(src, "rb").read()
    with P.Pod5File(src) as f:
        o, ln = [(o, ln) for n, o, ln in f.embedded if n == "reads"][0]
    r = ipc.open_file(pa.BufferReader(raw[o:o + ln]))
    lists, batches, k = [], [], 0
    for i in range(r.num_record_batches):
        b = r.get_batch(i)
        lists += b.column("signal").to_pylist()
        batches.append(list(range(k, k + b.num_rows)))
        k += b.num_rows
    return lists, batches


def _expected(lists, batches, status):
    """the reference's writes: (kept reads, kept rows in order, orphan rows)"""
    kept_reads, kept_rows, orphans = [], set(), 0
    for batch in batches:
        for r in batch:
            bad = [i for i, row in enumerate(lists[r]) if status[row]]
            if bad:
                kept_rows.update(lists[r][:bad[0]])
                orphans += bad[0]
                break
            kept_reads.append(r)
            kept_rows.update(lists[r])
    return kept_reads, sorted(kept_rows), orphans


def _nan_safe(v):
    return ["nan" if isinstance(x, float) and x != x else x for x in v]


def _check(src, out, status, res):
    lists, batches = _reads_rows(src)
    kept_reads, kept_rows, orphans = _expected(lists, batches, status)
    with P.Pod5File(src) as f:
        t = f.signal_table()
    with P.Pod5File(out) as g:
        u = g.signal_table()
        assert g.rows == len(kept_rows)
    remap = {old: new for new, old in enumerate(kept_rows)}
    for new, old in enumerate(kept_rows):
        assert u.blob(new) == t.blob(old) and u.samples[new] == t.samples[old]
        assert bytes(u.read_ids[new]) == bytes(t.read_ids[old])
    a, b = _tables(src)["reads"], _tables(out)["reads"]
    assert b.num_rows == len(kept_reads)
    assert b.schema.equals(a.schema, check_metadata=True)
    sub = a.take(pa.array(kept_reads, pa.int64()))
    for name in a.column_names:
        if name == "signal":
            assert b.column(name).to_pylist() == [[remap[x] for x in sub.column(name)[i].as_py()]
                                                  for i in range(len(kept_reads))]
        else:
            assert _nan_safe(b.column(name).to_pylist()) == _nan_safe(sub.column(name).to_pylist()), name
    assert _tables(out)["run_info"].equals(_tables(src)["run_info"])
    assert res["dropped_rows"] == len(status) - len(kept_rows)
    assert res["dropped_reads"] == len(lists) - len(kept_reads)
    assert res["orphan_rows"] == orphans


@pytest.mark.parametrize("per_batch", [None, 3])
def test_no_failure_is_the_plain_file(tmp_path, per_batch):
    src = FIXTURE if per_batch is None else _rebatched(tmp_path, per_batch)
    mk = bytes(range(16))
    with P.Pod5File(src) as f:
        t = f.signal_table()
        a, b = str(tmp_path / "a.pod5"), str(tmp_path / "b.pod5")
        P.write_pod5(a, t, source=f, section_marker=mk)
        res = P.write_pod5_keep_going(b, t, np.zeros(t.rows, np.int32), source=f, section_marker=mk)
    assert open(a, "rb").read() == open(b, "rb").read()
    assert res["dropped_rows"] == 0 and res["first_failed_row"] is None


def test_failure_drops_the_rest_of_the_read_batch(tmp_path):
    lists, _ = _reads_rows(FIXTURE)
    k = next(i for i, rows in enumerate(lists) if len(rows) >= 2)
    status = np.zeros(22, np.int32)
    status[lists[k][1]] = 1  # the read's second chunk: its first stays, an orphan
    out = str(tmp_path / "kg.pod5")
    with P.Pod5File(FIXTURE) as f:
        res = P.write_pod5_keep_going(out, f.signal_table(), status, source=f)
    _check(FIXTURE, out, status, res)
    assert res["orphan_rows"] == 1 and res["failed_batches"] == 1 and res["first_status"] == 1


def test_failures_in_several_read_batches(tmp_path):
    src = _rebatched(tmp_path, 3)
    lists, batches = _reads_rows(src)
    assert len(batches) == 4
    status = np.zeros(22, np.int32)
    status[lists[batches[1][1]][0]] = 9   # batch 1: its second read fails at its first chunk
    status[lists[batches[3][0]][-1]] = 1  # batch 3: its first read fails at its last chunk
    out = str(tmp_path / "kg.pod5")
    with P.Pod5File(src) as f:
        res = P.write_pod5_keep_going(out, f.signal_table(), status, source=f, rows_per_batch=5)
    _check(src, out, status, res)
    assert res["failed_batches"] == 2
    with P.Pod5File(out) as g:  # our own reader takes it back, record batches of 5 rows
        assert g.batches == -(-g.rows // 5)


def test_without_reads_table_rows_drop_alone(tmp_path):
    with P.Pod5File(FIXTURE) as f:
        t = f.signal_table()
    src = str(tmp_path / "bare.pod5")
    P.write_pod5(src, t)
    status = np.zeros(22, np.int32)
    status[[3, 4, 17]] = 1
    out = str(tmp_path / "kg.pod5")
    with P.Pod5File(src) as f:
        res = P.write_pod5_keep_going(out, f.signal_table(), status, source=f)
    assert res["dropped_rows"] == 3 and res["first_failed_row"] == 3
    with P.Pod5File(out) as g:
        u = g.signal_table()
    kept = [i for i in range(22) if not status[i]]
    assert [u.blob(i) for i in range(u.rows)] == [t.blob(i) for i in kept]


def test_unlisted_failing_row_is_reported(tmp_path):
    """A row no read lists (here a 23rd signal row behind the fixture's reads table) that fails is
    dropped and reported in first_failed_row / first_status like a listed one."""
    with P.Pod5File(FIXTURE) as f:
        t = f.signal_table()
        extra = P.SignalTable(np.concatenate([t.read_ids, t.read_ids[:1]]), np.concatenate([t.samples, t.samples[:1]]),
                              np.concatenate([t.offsets, [t.offsets[-1] + (t.offsets[1] - t.offsets[0])]]).astype(np.uint64),
                              np.concatenate([t.data, t.data[t.offsets[0]:t.offsets[1]]]), t.signal_type)
        src = str(tmp_path / "extra.pod5")
        P.write_pod5(src, extra, source=f)
    status = np.zeros(23, np.int32)
    status[22] = 7
    out = str(tmp_path / "kg.pod5")
    with P.Pod5File(src) as f:
        res = P.write_pod5_keep_going(out, f.signal_table(), status, source=f)
    assert res["dropped_rows"] == 1 and res["dropped_reads"] == 0
    assert res["first_failed_row"] == 22 and res["first_status"] == 7
    with P.Pod5File(out) as g:
        assert g.rows == 22


def test_null_data_is_an_invalid_argument(tmp_path):
    import ctypes as C

    from rawnanoporesignalcompression_amd import _native

    lib = _native.load()
    with P.Pod5File(FIXTURE) as f:
        t = f.signal_table()
        st = np.zeros(t.rows, np.int32)
        ids = np.ascontiguousarray(t.read_ids)
        rc = lib.pgn_pod5_write_file_keep_going(str(tmp_path / "x.pod5").encode(), f._h, 2, t.rows,
                                                ids.ctypes.data, t.samples.ctypes.data, t.offsets.ctypes.data, None,
                                                st.ctypes.data, 100, None, None)
    assert rc == 10  # PGN_ERR_INVALID_ARG
    assert not (tmp_path / "x.pod5").exists()
