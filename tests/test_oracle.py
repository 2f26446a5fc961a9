"""The oracle (tests' checker) pinned against the reference's own fixtures and known answers."""
import hashlib

import numpy as np
import pytest

import _oracle as O
from _golden import c5_blobs, golden, real_vbz_chunks


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_libzstd_release_line():
    v = O.oracle().pgno_zstd_version()
    assert 10400 <= v < 10500, v  # libzstd 1.4.x (the reference's conda `zstd` era)


def test_vbz_reencode_of_reference_fixture_is_byte_identical():
    """pod5/test_data/multi_fast5_zip_v3.pod5 (written by the pod5 tooling): decoding every signal
    chunk with the VBZ restatement and re-encoding it reproduces the fixture bytes exactly."""
    chunks = real_vbz_chunks()
    assert len(chunks) == 22 and sum(n for _, n in chunks) == 1_548_931
    for vbz, n in chunks:
        rc, x = O.vbz_decompress(vbz, n)
        assert rc == 0
        assert O.vbz_compress(x) == vbz


def test_c5_real_fixture_goldens_and_ratio():
    g = golden()
    tot = 0
    for (vbz, n), meta in zip(real_vbz_chunks(), g["real"]):
        _, x = O.vbz_decompress(vbz, n)
        assert sha(x.tobytes()) == meta["signal_sha256"]
        rc, blob, st = O.c5_compress(x)
        assert rc == 0 and sha(blob) == meta["c5_sha256"]
        assert [int(v) for v in st] == meta["streams"]
        rc, back = O.c5_decompress(blob, n)
        assert rc == 0 and np.array_equal(back, x)
        tot += len(blob)
    # the compiled reference measured 6.640 (C5) vs 6.750 (VBZ) bits/sample here
    assert round(8.0 * tot / 1_548_931, 3) == 6.640
    assert round(g["real_totals"]["vbz_bits_per_sample"], 2) == 6.75


def test_committed_blobs_decode():
    blobs = c5_blobs()
    rc, x = O.c5_decompress(blobs["synth_small"], 3000)
    assert rc == 0 and np.array_equal(x, O.synth_read(7, 3000))


def test_synth_generator_known_answers():
    for s in golden()["synth"]:
        x = O.synth_read(s["read"], s["samples"])
        assert sha(x.tobytes()) == s["signal_sha256"]
        rc, blob, _ = O.c5_compress(x)
        assert sha(blob) == s["c5_sha256"]


def test_c5_stream_layout_by_hand():
    """encode_scalar_N01 (C5.hpp:57-152) on a hand-checked input."""
    x = np.array([0, 1, -1, 20, 20, 400, 400 - 300, 5], np.int16)
    keys = np.zeros(2, np.uint8)
    S, M, Ll, Lh = (np.zeros(8, np.uint8) for _ in range(4))
    sizes = np.zeros(5, np.uint64)
    O.oracle().pgno_c5_split(x.ctypes.data, x.size, keys.ctypes.data, S.ctypes.data, M.ctypes.data,
                             Ll.ctypes.data, Lh.ctypes.data, sizes.ctypes.data)
    # deltas 0,1,-2,21,0,380,-300,-95 -> zz 0,2,3,42,0,760,599,189
    # codes: 0, 1(S 1), 1(S 2), 2(M 25), 0, 3(L 487=0x1E7), 3(L 326=0x146), 2(M 172)
    assert list(sizes) == [2, 1, 2, 2, 2]
    assert keys[0] == (0 | 1 << 2 | 1 << 4 | 2 << 6) and keys[1] == (0 | 3 << 2 | 3 << 4 | 2 << 6)
    assert S[0] == (1 | 2 << 4)
    assert list(M[:2]) == [25, 172]
    assert list(Ll[:2]) == [0xE7, 0x46] and list(Lh[:2]) == [1, 1]


def test_edge_and_error_behaviour():
    for e in golden()["edge"]:
        x = O.synth_read(1000 + e["samples"], e["samples"])
        rc, blob, _ = O.c5_compress(x)
        assert rc == e["status"] == 0 and sha(blob) == e["c5_sha256"]
    # empty chunk: five empty 9-byte frames behind four prefixes (C5.hpp:429-462)
    rc, blob, _ = O.c5_compress(np.zeros(0, np.int16))
    assert rc == 0 and len(blob) == 4 * 8 + 5 * 9
    # uniform int16 overflows max(2n+26, 1024) (C5.hpp:420-427)
    x = np.random.default_rng(0).integers(-32768, 32768, 100_000).astype(np.int16)
    rc, required, _ = O.c5_compress(x)
    assert rc == O.DST_TOO_SMALL and required > 2 * 100_000 + 26
    # decode statuses (C5.hpp:495-502, 593-600, 675-677)
    x = O.synth_read(3, 5000)
    _, blob, _ = O.c5_compress(x)
    # n - 1 leaves the key length and (unless the last code is 3) the Lhigh walk unchanged: the
    # reference accepts it; a shorter key stream shifts every stream start and fails the check
    assert O.c5_decompress(blob, 4999)[0] == 0
    assert O.c5_decompress(blob, 4000)[0] in (O.REMAINING, O.CORRUPT)
    assert O.c5_decompress(blob[:8] + b"\0" + blob[9:], 5000)[0] == O.NOT_ZSTD
    assert O.c5_decompress(blob[:-3], 5000)[0] == O.ZSTD_DECOMPRESS


def test_c5_blob_from_other_encoder_settings_round_trips():
    """The assembled blobs the GPU decoder test uses: the oracle (libzstd reader) inverts them."""
    for level, wlog in [(3, 0), (19, 0), (1, 10), (19, 11)]:
        x = O.synth_read(77 + level, 30000)
        blob = O.c5_assemble([O.zstd_compress_ex(s, level, wlog) for s in O.c5_streams(x)])
        rc, back = O.c5_decompress(blob, x.size)
        assert rc == 0 and np.array_equal(back, x), (level, wlog)
