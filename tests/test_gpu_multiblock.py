"""GPU parity of multi-block zstd frames (streams above one 128 KiB block): C5 chunks up to and above
the batched passes' 262,144 samples (the large-chunk pass, up to PGN_MAX_CHUNK_SAMPLES), noisy VBZ /
C1 chunks whose svb16 buffer exceeds one block, and frames above 512 KiB (windowLog 19 < source:
window-descriptor frames whose matches stay inside the window).  The reference's ZSTD_compress
takes any size (signal_compression.cpp:57-66, C5.hpp:337-413).  Frames equal libzstd 1.4.x's byte
for byte (through the oracle) and round-trip, per chunk and batched.  Needs an MI355X."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

MAX = 262144


def _noisy(n, seed, sd):
    rng = np.random.default_rng(seed)
    return np.clip(np.round(rng.normal(0, sd, n)), -32768, 32767).astype(np.int16)


def _c5_signals():
    sig = {f"synth_{n}": O.synth_read(7000 + n, n) for n in (131073, 150000, 200000, 262143, MAX)}
    sig["noisy_200000"] = _noisy(200000, 1, 40)            # M stream ~200 KB: two blocks, table repeat
    sig["steps_240000"] = np.repeat(np.random.default_rng(2).integers(300, 700, 4000),
                                    60)[:240000].astype(np.int16)  # long matches across blocks
    sig["zeros_then_noise"] = np.concatenate([np.zeros(140000, np.int16), _noisy(100000, 3, 12)])
    return sig


def test_c5_large_chunks_identical(codec):
    for name, x in _c5_signals().items():
        rc, ref, _ = O.c5_compress(x)
        if rc != 0:  # wider than max(2n+26, 1024): the reference refuses it too
            continue
        assert codec.compress_signal(x) == ref, name
        assert np.array_equal(codec.decompress_signal(ref, sample_count=x.size), x), name


def test_c5_over_limit_is_unsupported(codec):
    from rawnanoporesignalcompression_amd import PGN_MAX_CHUNK_SAMPLES, PGNanoError

    x = np.zeros(PGN_MAX_CHUNK_SAMPLES + 1, np.int16)
    with pytest.raises(PGNanoError) as ei:
        codec.compress_signal(x)
    assert ei.value.status == 9


BIG = [MAX + 1, 300000, 600000, 1048576]


@pytest.mark.parametrize("n", BIG)
def test_c5_chunks_above_batched_pass(codec, n):
    """Chunks above 262,144 samples (the large-chunk pass); from 524,289 samples the M/L streams
    are frames above 512 KiB (window descriptor, windowed matches)."""
    for x in (O.synth_read(9000 + n, n), _noisy(n, n, 25)):
        rc, ref, _ = O.c5_compress(x)
        assert rc == 0
        assert codec.compress_signal(x) == ref, n
        assert np.array_equal(codec.decompress_signal(ref, sample_count=x.size), x), n


def test_c5_long_range_repeats_outside_window(codec):
    """A stream whose repeats lie 600,000 bytes back (beyond the 512 KiB window) and 400,000 bytes
    back (inside it): libzstd matches only the latter."""
    base = _noisy(400000, 31, 30)
    x = np.concatenate([base, _noisy(200000, 32, 30), base[:300000], base[100000:400000]])
    rc, ref, _ = O.c5_compress(x)
    assert rc == 0
    assert codec.compress_signal(x) == ref
    assert np.array_equal(codec.decompress_signal(ref, sample_count=x.size), x)


@pytest.mark.parametrize("big", [False, True])
def test_c5_batch_mixed_sizes(codec, big):
    import torch

    rng = np.random.default_rng(21)
    counts = rng.integers(100000, MAX + 1, 96).astype(np.int32)
    counts[:4] = [131072, 131073, MAX, 7]
    if big:  # chunks for the large-chunk pass among the batched ones (the last call's buffers are reused)
        counts[[5, 17, 40, 41, 95]] = [MAX + 1, 1048576, 700000, 300001, 2000000]
    samples, offs, cnt = codec.synth_reads(len(counts), counts, seed=42)
    enc = codec.compress_batch(samples, offs, cnt)
    out, _, st = codec.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cnt)
    torch.cuda.synchronize()
    assert (enc.status == 0).all() and (st == 0).all()
    assert torch.equal(out, samples)
    blobs = enc.blobs.cpu().numpy()
    bo, bs = enc.offsets.cpu().numpy(), enc.sizes.cpu().numpy()
    for r in list(range(0, len(counts), 7)) + [1, 2] + ([5, 17, 40, 41, 95] if big else []):
        rc, ref, _ = O.c5_compress(O.synth_read(r, int(counts[r])))
        assert rc == 0 and blobs[bo[r]:bo[r] + bs[r]].tobytes() == ref, (r, int(counts[r]))


@pytest.fixture(scope="module")
def vbz():
    from rawnanoporesignalcompression_amd import VBZCodec

    c = VBZCodec(0)
    yield c
    c.close()


def test_vbz_noisy_default_chunk(vbz):
    """A noisy 102,400-sample chunk: its svb16 buffer (> 128 KiB) is a two-block frame."""
    import torch

    xs = [_noisy(102400, s, sd) for s, sd in ((4, 300), (5, 3000), (6, 20000))]
    xs.append(np.random.default_rng(7).integers(-32768, 32768, 102400).astype(np.int16))
    for i, x in enumerate(xs):
        ref = O.vbz_compress(x)
        assert vbz.compress_signal(x) == ref, i
        assert np.array_equal(vbz.decompress_signal(ref, sample_count=x.size), x), i
    flat = np.concatenate(xs)
    dev = torch.device("cuda", 0)
    samples = torch.from_numpy(flat).to(dev)
    counts = torch.full((len(xs),), 102400, dtype=torch.int32, device=dev)
    offs = torch.arange(len(xs), dtype=torch.int64, device=dev) * 102400
    enc = vbz.compress_batch(samples, offs, counts)
    out, _, st = vbz.decompress_batch(enc.blobs, enc.offsets, enc.sizes, counts)
    torch.cuda.synchronize()
    assert (enc.status == 0).all() and (st == 0).all() and torch.equal(out, samples)
    blobs = enc.blobs.cpu().numpy()
    bo, bs = enc.offsets.cpu().numpy(), enc.sizes.cpu().numpy()
    for i, x in enumerate(xs):
        assert blobs[bo[i]:bo[i] + bs[i]].tobytes() == O.vbz_compress(x), i


@pytest.mark.parametrize("n", [240000, MAX, 400000, 1000000])
def test_vbz_svb16_above_512k(vbz, n):
    """Uniform noise: svb16 buffers of ~2.1 n bytes -- 510,000 B (four blocks, single segment) up to
    2.1 MB (window-descriptor frames, above the batched pass from 262,145 samples)."""
    x = np.random.default_rng(n).integers(-32768, 32768, n).astype(np.int16)
    ref = O.vbz_compress(x)
    assert vbz.compress_signal(x) == ref
    assert np.array_equal(vbz.decompress_signal(ref, sample_count=x.size), x)


def test_vbz_batch_with_large_chunks(vbz):
    import torch

    rng = np.random.default_rng(77)
    xs = [rng.integers(-32768, 32768, n).astype(np.int16) for n in (102400, 400000, 5000, MAX + 10)]
    xs.append(_noisy(1200000, 78, 400))
    flat = np.concatenate(xs)
    dev = torch.device("cuda", 0)
    counts_np = np.array([x.size for x in xs], np.int64)
    samples = torch.from_numpy(flat).to(dev)
    counts = torch.from_numpy(counts_np.astype(np.int32)).to(dev)
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(counts_np)[:-1]])).to(dev)
    enc = vbz.compress_batch(samples, offs, counts)
    out, _, st = vbz.decompress_batch(enc.blobs, enc.offsets, enc.sizes, counts)
    torch.cuda.synchronize()
    assert (enc.status == 0).all() and (st == 0).all() and torch.equal(out, samples)
    blobs = enc.blobs.cpu().numpy()
    bo, bs = enc.offsets.cpu().numpy(), enc.sizes.cpu().numpy()
    for i, x in enumerate(xs):
        assert blobs[bo[i]:bo[i] + bs[i]].tobytes() == O.vbz_compress(x), i


def test_c1_large_data_frame():
    from rawnanoporesignalcompression_amd import PGNanoCodec

    c = PGNanoCodec(0, variant="C1")
    try:
        for i, x in enumerate([_noisy(102400, 10, 3000), O.synth_read(11, 200000), _noisy(400000, 12, 3000)]):
            rc, ref, _ = O.variant_compress("C1", x)
            assert rc == O.OK
            assert c.compress_signal(x) == ref, i
            assert np.array_equal(c.decompress_signal(ref, sample_count=x.size), x), i
    finally:
        c.close()
