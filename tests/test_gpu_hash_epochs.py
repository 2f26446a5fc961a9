"""GPU parity across the match search's hash-table epochs (csrc/pgn_zenc.h, ht_next_epoch): a slot's
table is never cleared between frames -- entries of another epoch's 5-bit tag read as empty -- and
when the tags run out (every 31 frames) only the extent written since the last clear is zeroed.
With one encode slot per CU every slot compresses tens of frames per launch, so the tags wrap
several times, over frames of different table sizes (hashLog 15 for streams up to 16 KiB, 13, 14)
and both entry layouts (17-bit index + 10-bit fingerprint; 20-bit index + 7-bit fingerprint for
frames above 128 KiB).  Every blob must equal the oracle's (libzstd 1.4.x level 1)."""
import os

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def few_slots():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rawnanoporesignalcompression_amd import PGNanoCodec

    old = os.environ.get("PGN_ENC_WG_PER_CU")
    os.environ["PGN_ENC_WG_PER_CU"] = "1"  # read once, when the context is created
    try:
        c = PGNanoCodec(0)
    finally:
        if old is None:
            del os.environ["PGN_ENC_WG_PER_CU"]
        else:
            os.environ["PGN_ENC_WG_PER_CU"] = old
    yield c
    c.close()


def _encode_and_check(c, counts, seed, **gen):
    import torch

    samples, offs, cnt = c.synth_reads(len(counts), counts, seed=seed, **gen)
    enc = c.compress_batch(samples, offs, cnt)
    torch.cuda.synchronize()
    assert (enc.status.cpu().numpy() == 0).all()
    host, offs_h = samples.cpu().numpy(), offs.cpu().numpy()
    blobs, bo, bs = enc.blobs.cpu().numpy(), enc.offsets.cpu().numpy(), enc.sizes.cpu().numpy()
    largest = 0  # the largest stream handed to a zstd frame
    for r in range(len(counts)):
        x = host[offs_h[r]:offs_h[r] + counts[r]]
        rc, ref, st = O.c5_compress(x)
        assert rc == 0
        assert blobs[bo[r]:bo[r] + bs[r]].tobytes() == ref, (seed, r, int(counts[r]))
        largest = max(largest, int(st[:5].max()))
    out, _, dst = c.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cnt)
    torch.cuda.synchronize()
    assert (dst.cpu().numpy() == 0).all()
    assert torch.equal(out[: samples.numel()], samples[: out.numel()])
    return largest


def test_epoch_wraps_mixed_table_sizes_identical(few_slots):
    rng = np.random.default_rng(5)
    k = 2048  # ~8 chunks = ~40 frames per slot per launch: every slot's tags wrap
    small = rng.integers(0, 30000, k).astype(np.int32)
    small[:4] = [0, 1, 7, 100000]
    _encode_and_check(few_slots, small, seed=101)
    # noisy chunks: the class-3 streams exceed 128 KiB (multi-block frames, 20-bit index layout); the
    # slots' tables keep the entries of the first launch under older tags
    big = np.full(300, 150000, dtype=np.int32)
    big[::7] = 200000
    assert _encode_and_check(few_slots, big, seed=202, noise_sd=400) > 131072
    # back to small frames over tables written in the other layout
    small2 = rng.integers(0, 30000, k).astype(np.int32)
    _encode_and_check(few_slots, small2, seed=303)
