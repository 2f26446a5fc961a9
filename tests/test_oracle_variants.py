"""The oracle's restatement of the other compile-time pgnano variants (C4, C1, C2, C3, VBZ0;
pgnano.cpp:70-92) -- hand-checked stream layouts, structural relations to the pinned C5/VBZ
restatements, round trips and error statuses.  The reference ships no test or fixture for any of
these variants, so their parity is pinned by these checks, not by reference output."""
import numpy as np
import pytest

import _oracle as O
from _golden import real_vbz_chunks

# deltas 0,1,-2,21,0,380,-300,-95 -> zig-zag 0,2,3,42,0,760,599,189
X = np.array([0, 1, -1, 20, 20, 400, 400 - 300, 5], np.int16)


def test_c4_layout_by_hand():
    """encode_scalar_N02 (C4.hpp:53-145): classes on the raw value, no offsets."""
    k, s, m, ll, lh = O.variant_streams("C4", X)
    # codes: 0, 1 (2), 1 (3), 2 (42), 0, 3 (760 = 0x2F8), 3 (599 = 0x257), 2 (189)
    assert k == bytes([0 | 1 << 2 | 1 << 4 | 2 << 6, 0 | 3 << 2 | 3 << 4 | 2 << 6])
    assert s == bytes([2 | 3 << 4])
    assert m == bytes([42, 189])
    assert ll == bytes([0xF8, 0x57]) and lh == bytes([2, 2])


def test_c1_is_svb16_split_in_two_frames():
    """compress_signal_KD (C1.hpp:202-285): the VBZ svb16 buffer (pinned by the fixture) cut at
    keys_length into a keys frame and a data frame."""
    k, d = O.variant_streams("C1", X)
    assert k == bytes([0b01100000])  # 760 and 599 take two bytes
    assert d == bytes([0, 2, 3, 42, 0, 0xF8, 0x02, 0x57, 0x02, 189])
    for vbz, n in real_vbz_chunks()[:5]:
        _, x = O.vbz_decompress(vbz, n)
        svb = np.zeros(3 * n + 16, np.uint8)
        m = O.oracle().pgno_vbz_svb_encode(x.ctypes.data, n, svb.ctypes.data)
        k, d = O.variant_streams("C1", x)
        assert k + d == svb[:m].tobytes()
        # the reference's own VBZ frame compresses the same bytes the two C1 frames split
        assert O.zstd_compress1(k + d) == vbz


def test_c2_c3_layout_by_hand():
    k2, lo, hi = O.variant_streams("C2", X)
    assert k2 == bytes([0b01100000])
    assert lo == bytes([0, 2, 3, 42, 0, 0xF8, 0x57, 189]) and hi == bytes([2, 2])
    k3, ll, lh, h = O.variant_streams("C3", X)
    assert k3 == k2
    assert ll == bytes([0, 2, 3, 42, 0, 189]) and lh == bytes([0xF8, 0x57]) and h == bytes([2, 2])


def test_vbz0_layout_by_hand():
    """encode_scalar_VBZ1 (VBZ_0.hpp:60-172): C5 classes/offsets, values as 1/2/4 nibbles."""
    (buf,) = O.variant_streams("VBZ0", X)
    keys = bytes([0 | 1 << 2 | 1 << 4 | 2 << 6, 0 | 3 << 2 | 3 << 4 | 2 << 6])
    # nibbles: 1 (2-1), 2 (3-1), 25 -> 9,1, 487=0x1E7 -> 7,E,1,0, 326=0x146 -> 6,4,1,0, 172=0xAC -> C,A
    nib = [1, 2, 9, 1, 7, 0xE, 1, 0, 6, 4, 1, 0, 0xC, 0xA]
    data = bytes(nib[i] | nib[i + 1] << 4 for i in range(0, len(nib), 2))
    assert buf == keys + data


@pytest.mark.parametrize("variant", ["C4", "C1", "C2", "C3", "VBZ0"])
def test_round_trip_and_frames(variant):
    sigs = [O.synth_read(i, n) for i, n in enumerate([0, 1, 2, 3, 4, 5, 7, 8, 9, 257, 1025, 20000, 102400])]
    sigs += [O.vbz_decompress(b, n)[1] for b, n in real_vbz_chunks()[:4]]
    for x in sigs:
        rc, blob, st = O.variant_compress(variant, x)
        assert rc == O.OK, (variant, x.size)
        rc, back = O.variant_decompress(variant, blob, x.size)
        assert rc == O.OK and np.array_equal(back, x), (variant, x.size)
        frames = [O.zstd_compress1(s) for s in O.variant_streams(variant, x)]
        assert len(frames) == O.VARIANT_FRAMES[variant]
        want = frames[0] if variant == "VBZ0" else O.variant_assemble(frames)
        assert blob == want
        nf = len(frames)
        assert [int(v) for v in st[5:5 + nf]] == [len(f) for f in frames]


def test_empty_chunk_blobs():
    # every frame of an empty stream is the 9-byte empty frame, behind nf-1 prefixes
    for v, nf in O.VARIANT_FRAMES.items():
        rc, blob, _ = O.variant_compress(v, np.zeros(0, np.int16))
        assert rc == O.OK and len(blob) == 8 * (nf - 1) + 9 * nf, v
        assert O.variant_decompress(v, blob, 0)[0] == O.OK


def test_capacity_and_decode_errors():
    x = np.random.default_rng(4).integers(-32768, 32768, 60000).astype(np.int16)
    for v in ["C4", "C1", "C2", "C3"]:
        rc, required, _ = O.variant_compress(v, x)
        assert rc == O.DST_TOO_SMALL and required > 2 * 60000 + 26, v
    assert O.variant_compress("VBZ0", x)[0] == O.ZSTD_COMPRESS  # ZSTD_compress into the span fails
    y = O.synth_read(3, 5000)
    for v in O.VARIANT_FRAMES:
        _, blob, _ = O.variant_compress(v, y)
        bad_magic = blob[:8] + b"\0" + blob[9:] if v != "VBZ0" else b"\0" + blob[1:]
        assert O.variant_decompress(v, bad_magic, 5000)[0] == O.NOT_ZSTD, v
        assert O.variant_decompress(v, blob[:-3], 5000)[0] == O.ZSTD_DECOMPRESS, v
        assert O.variant_decompress(v, blob, 4000)[0] in (O.REMAINING, O.CORRUPT), v
