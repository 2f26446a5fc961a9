"""A frame's first block whose sequences are one batch (<= 64; the C5 Lhigh frame) is checked at once and
executed in LDS when its output fits 4 KiB, else by global copies (pgn_zdec.h exec_one_batch).  Its
statuses and samples must be the oracle's (libzstd's ZSTD_decompress, C5.hpp:588-677): valid frames
whose matches repeat a short period (the in-LDS pattern copy), blocks too large for LDS, and Lhigh frames
with their sequence section corrupted byte by byte (literal runs past the section, matches before the
frame start, outputs past the claimed content size, a bitstream not consumed to its first bit)."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


def _lhigh_start(blob: bytes) -> int:
    """Offset of the fifth (Lhigh) frame: behind four length-prefixed frames (C5.hpp:429-462)."""
    p = 0
    for _ in range(4):
        p += 8 + int.from_bytes(blob[p:p + 8], "little")
    return p


def _decode(codec, blobs, lens):
    import torch

    dev = torch.device("cuda", 0)
    data = b"".join(blobs)
    bsz = np.array([len(b) for b in blobs], np.int64)
    boff = np.concatenate([[0], np.cumsum(bsz)[:-1]]).astype(np.int64)
    din = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(dev)
    out, _, st = codec.decompress_batch(din, torch.from_numpy(boff).to(dev), torch.from_numpy(bsz).to(dev),
                                        torch.from_numpy(np.asarray(lens, np.int32)).to(dev))
    torch.cuda.synchronize()
    return out.cpu().numpy(), st.cpu().numpy()


def _check(codec, blobs, lens):
    out, st = _decode(codec, blobs, lens)
    so = np.concatenate([[0], np.cumsum(np.asarray(lens, np.int64))])
    nbad = 0
    for i, b in enumerate(blobs):
        rc, ref = O.c5_decompress(b, int(lens[i]))
        if rc == 0 and st[i] == 3 and not O.c5_frames_strictly_valid(b):
            continue  # libzstd's double-symbol Huffman decoder accepts one trailing codeword
        assert st[i] == rc, (i, rc, st[i])
        nbad += rc != 0
        if rc == 0:
            assert np.array_equal(out[so[i]:so[i + 1]], ref), i
    return nbad


def _periodic(n, period, amp, seed):
    rng = np.random.default_rng(seed)
    pat = rng.integers(-amp, amp, period)
    return np.resize(pat, n).astype(np.int16)


@pytest.mark.parametrize("batch", [40, 300])  # the small-batch (cooperative) and the batch decoder
def test_one_batch_blocks_valid_and_corrupted(codec, batch):
    rng = np.random.default_rng(17 + batch)
    reads, lens = [], []
    for i in range(batch):
        k = i % 5
        if k == 0:    # the C5 bench shape: Lhigh ~1.2 KB, ~18 sequences
            x = O.synth_read(9000 + i, 100000)
        elif k == 1:  # large deltas with a short period: Lhigh matches that repeat a period < 64
            x = _periodic(int(rng.integers(500, 3000)), int(rng.integers(2, 9)), 20000, i)
        elif k == 2:  # the same past 4 KiB of Lhigh output: the global-copy branch
            x = _periodic(int(rng.integers(6000, 20000)), int(rng.integers(2, 40)), 20000, i)
        elif k == 3:  # class-3 runs between noise
            x = O.synth_read(9000 + i, 30000, noise_sd=900)
        else:         # short reads
            x = O.synth_read(9000 + i, int(rng.integers(64, 4000)))
        reads.append(x)
        lens.append(x.size)
    blobs = []
    for x in reads:
        rc, b, _ = O.c5_compress(x)
        assert rc == 0
        blobs.append(b)
    assert _check(codec, blobs, lens) == 0
    # corrupt the Lhigh frame's tail (its sequence section sits at the frame's end)
    bad = []
    for i, b in enumerate(blobs):
        bb = bytearray(b)
        s = _lhigh_start(b)
        span = len(bb) - s
        if span > 12:
            j = len(bb) - 1 - int(rng.integers(0, min(span - 8, 48)))
            bb[j] ^= int(rng.integers(1, 256))
        bad.append(bytes(bb))
    assert _check(codec, bad, lens) > 0
