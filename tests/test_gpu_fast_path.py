"""The batch decoder's fast frame path (pgn_zdec.h dec_frame_fast) and its fall-through to the general
frame decoder, against the oracle (libzstd's ZSTD_decompress as C5.hpp:520-600 calls it).

dec_zstd_kernel decodes a frame that is one raw last block, or one compressed last block of literals
only with four Huffman streams and a new table (turned into a dec_huf_kernel job on the deferred path),
inline; anything else -- a skippable frame after the frame, a dictionary-id field, trailing bytes,
frames from other encoder settings -- must reach the general decoder and end with the oracle's status
and samples.  Each variant is applied to every one of a chunk's five frames in turn, in batches that
take the batch path (more than 64 chunks) with and without the deferred Huffman sections.
"""
import os

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dcodec():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rawnanoporesignalcompression_amd import PGNanoCodec

    keys = ("PGN_DEFER_MIN_CHUNKS", "PGN_DEFER_G")
    old = {k: os.environ.get(k) for k in keys}
    os.environ["PGN_DEFER_MIN_CHUNKS"] = "1"
    os.environ["PGN_DEFER_G"] = "128"
    try:
        c = PGNanoCodec(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    yield c
    c.close()


def _decode(codec, blobs, lens):
    import torch

    dev = torch.device("cuda", 0)
    sizes = np.array([len(b) for b in blobs], np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    flat = np.frombuffer(b"".join(bytes(b) for b in blobs), np.uint8).copy()
    counts = np.asarray(lens, np.int32)
    out, _, st = codec.decompress_batch(torch.from_numpy(flat).to(dev), torch.from_numpy(offs).to(dev),
                                        torch.from_numpy(sizes).to(dev), torch.from_numpy(counts).to(dev))
    torch.cuda.synchronize()
    so = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    o = out.cpu().numpy()
    return [o[so[i]:so[i + 1]] for i in range(len(lens))], st.cpu().numpy()


def _skippable(frame: bytes) -> bytes:
    return frame + (0x184D2A53).to_bytes(4, "little") + (5).to_bytes(4, "little") + b"abcde"


def _dict_id(frame: bytes, did: int) -> bytes:
    """the same frame with a one-byte dictionary-id field (0: accepted, else an error)"""
    f = bytearray(frame)
    f[4] |= 1
    return bytes(f[:5]) + bytes([did]) + bytes(f[5:])


def _trailing(frame: bytes) -> bytes:
    return frame + b"\x00"


VARIANTS = {
    "skippable": _skippable,
    "dict_id_0": lambda f: _dict_id(f, 0),
    "dict_id_7": lambda f: _dict_id(f, 7),
    "trailing_byte": _trailing,
}


def _cases():
    xs = [O.synth_read(700 + i, n) for i, n in enumerate([4000, 20000, 65536, 100000])]
    blobs, lens = [], []
    for x in xs:
        frames = [O.zstd_compress1(s) for s in O.c5_streams(x)]
        blobs.append(O.c5_assemble(frames))
        lens.append(x.size)
        for fn in VARIANTS.values():
            for k in range(5):
                fr = list(frames)
                fr[k] = fn(fr[k])
                blobs.append(O.c5_assemble(fr))
                lens.append(x.size)
        for level, wlog in ((3, 0), (19, 0), (-5, 0), (1, 10)):
            blobs.append(O.c5_assemble([O.zstd_compress_ex(s, level, wlog) for s in O.c5_streams(x)]))
            lens.append(x.size)
    return blobs, lens


@pytest.mark.parametrize("deferred", [False, True])
def test_fast_path_fall_through_equals_oracle(codec, dcodec, deferred):
    blobs, lens = _cases()
    assert len(blobs) > 64  # the batch path
    c = dcodec if deferred else codec
    got, st = _decode(c, blobs, lens)
    if deferred:
        assert "dec_huf_kernel" in c.kernels(1)
    for i, b in enumerate(blobs):
        rc, ref = O.c5_decompress(b, int(lens[i]))
        assert st[i] == rc, (i, rc, st[i])
        if rc == 0:
            assert np.array_equal(got[i], ref), i
    assert (st == 0).sum() > len(blobs) // 2  # most variants decode (skippable frames, dictionary id 0)
