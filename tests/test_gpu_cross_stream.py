"""Keys that claim more S, M or class-3 samples than those streams hold, through the batch decode path,
against the oracle's merge over the concatenated intermediate (C5.hpp:173-257 as driven by
C5.hpp:600-677).

The reference reads the five decoded streams as one buffer, so such keys read on into the next
stream's bytes (and "Remaining data" / an out-of-bounds read decide the status).  Blobs are built here
from hand-made streams that do exactly that -- S reading into M, M into Llow, Llow into Lhigh -- with
random S / M / Llow bytes (raw blocks); they go through the batch path (more than 64 chunks) beside
ordinary chunks, and statuses and samples must equal the oracle's.  (Written for an experiment that
read raw S / Llow frames in place in the blob -- slower, not adopted, DESIGN.md §7 -- and kept: the
cross-stream reads are the reference's own semantics and no other test makes them succeed.)
"""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


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


def _keys(classes):
    c = np.asarray(classes, np.uint8)
    c = np.concatenate([c, np.zeros((-c.size) % 4, np.uint8)]).reshape(-1, 4)
    return (c[:, 0] | (c[:, 1] << 2) | (c[:, 2] << 4) | (c[:, 3] << 6)).astype(np.uint8).tobytes()


def _blob(rng, classes, dS, dM, dLl, dLh):
    streams = [_keys(classes)] + [rng.integers(0, 256, d, dtype=np.uint8).tobytes() for d in (dS, dM, dLl, dLh)]
    return O.c5_assemble([O.zstd_compress1(s) for s in streams])


def _raw_frame(frame: bytes) -> bool:
    """libzstd stored the stream as one raw block"""
    fhd = frame[4]
    ss, fcsf = (fhd >> 5) & 1, fhd >> 6
    hs = 5 + (0 if ss else 1) + ((1 if ss else 0) if fcsf == 0 else (1 << fcsf))
    bh = int.from_bytes(frame[hs:hs + 3], "little")
    return (bh & 7) == 1


def _cases(rng):
    """(n, blob); Lhigh holds exactly the class-3 samples' bytes, so that over-reads which stay inside
    the buffer end with the reference's status 0 and their samples are compared"""
    n = 4000
    out = []
    # S past dS into M: every sample class 1 needs n / 2 S bytes
    out.append((n, _blob(rng, [1] * n, 1000, 3000, 300, 0)))
    out.append((n, _blob(rng, [1] * n, 1999, 2500, 40, 0)))
    # M past dM into the raw Llow
    out.append((n, _blob(rng, [2] * n, 200, 3000, 1200, 0)))
    out.append((n, _blob(rng, [2] * (n - 100) + [3] * 100, 300, 3800, 400, 100)))
    # Llow past dLl into Lhigh
    out.append((n, _blob(rng, [3] * n, 300, 300, 2000, 4000)))
    # past the buffer (the reference's out-of-bounds read: PGN_ERR_CORRUPT) and "Remaining data"
    out.append((n, _blob(rng, [2] * n, 200, 3000, 900, 0)))
    out.append((n, _blob(rng, list(rng.integers(0, 4, n)), 600, 1000, 700, 2500)))
    # mixed classes, streams exactly as long as the keys need (the ordinary case, raw S / Llow)
    cl = rng.integers(0, 4, n)
    out.append((n, _blob(rng, cl, (int((cl == 1).sum()) + 1) // 2, int((cl == 2).sum()), int((cl == 3).sum()),
                         int((cl == 3).sum()))))
    return out


def test_cross_stream_reads_equal_oracle(codec):
    rng = np.random.default_rng(11)
    cases = _cases(rng)
    blobs, lens = [b for _, b in cases], [n for n, _ in cases]
    # the crafted S / Llow streams are raw frames
    for b in blobs:
        pos = 0
        frames = []
        for s in range(5):
            fl = int.from_bytes(b[pos:pos + 8], "little") if s < 4 else len(b) - pos
            pos += 8 if s < 4 else 0
            frames.append(b[pos:pos + fl])
            pos += fl
        assert _raw_frame(frames[1]) and _raw_frame(frames[3])
    # ordinary chunks around them: a batch of more than 64 chunks takes the batch path
    for i in range(70):
        x = O.synth_read(500 + i, int(rng.integers(1000, 30000)))
        rc, b, _ = O.c5_compress(x)
        assert rc == 0
        blobs.append(b)
        lens.append(x.size)
    got, st = _decode(codec, blobs, lens)
    for i, b in enumerate(blobs):
        rc, ref = O.c5_decompress(b, int(lens[i]))
        assert st[i] == rc, (i, rc, st[i])
        if rc == 0:
            assert np.array_equal(got[i], ref), i
    assert [int(s) for s in st[:5]] == [0] * 5  # over-reads that the reference accepts
