"""GPU parity of the other compile-time pgnano variants (C4, C1, C2, C3, VBZ0; pgnano.cpp:70-92) as a
runtime choice, through the C ABI (pgn_variant_*): byte-identical blobs and bit-exact samples against
the oracle restatement (tests/test_oracle_variants.py).  Needs an MI355X."""
import numpy as np
import pytest

import _oracle as O
from _golden import real_vbz_chunks
from test_gpu_parity import _pattern_signals

pytestmark = pytest.mark.gpu
VARIANTS = ["C4", "C1", "C2", "C3", "VBZ0"]


@pytest.fixture(scope="module")
def codecs():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rawnanoporesignalcompression_amd import PGNanoCodec

    cs = {v: PGNanoCodec(0, variant=v) for v in VARIANTS}
    yield cs
    for c in cs.values():
        c.close()


@pytest.mark.parametrize("variant", VARIANTS)
def test_real_chunks_and_edge_sizes_identical(codecs, variant):
    """The reference fixture's 22 chunks and the size thresholds: same bytes as the oracle, exact
    round trip."""
    c = codecs[variant]
    sigs = [O.vbz_decompress(b, n)[1] for b, n in real_vbz_chunks()]
    sigs += [O.synth_read(3000 + n, n) for n in [0, 1, 2, 3, 4, 5, 7, 8, 9, 255, 256, 257, 1023, 1024, 1025, 16385,
                                                 65792, 102400, 131072, 131073, 200000, 262144]]

    for i, x in enumerate(sigs):
        rc, ref, _ = O.variant_compress(variant, x)
        assert rc == O.OK
        blob = c.compress_signal(x)  # streams above 128 KiB: multi-block frames
        assert blob == ref, (variant, i, x.size)
        assert np.array_equal(c.decompress_signal(blob, sample_count=x.size), x), (variant, i)


@pytest.mark.parametrize("variant", VARIANTS)
def test_pattern_signals(codecs, variant):
    from rawnanoporesignalcompression_amd import PGNanoError

    c = codecs[variant]
    for name, x in _pattern_signals().items():
        rc, ref, _ = O.variant_compress(variant, x)
        if rc == O.OK:  # streams above 128 KiB included (multi-block frames)
            assert c.compress_signal(x) == ref, (variant, name)
        else:
            with pytest.raises(PGNanoError) as ei:
                c.compress_signal(x)
            assert ei.value.status == rc, (variant, name)
        if rc == O.OK:
            assert np.array_equal(c.decompress_signal(ref, sample_count=x.size), x), (variant, name)


@pytest.mark.parametrize("variant", VARIANTS)
def test_batch_identical_stats_round_trip(codecs, variant):
    import torch

    c = codecs[variant]
    rng = np.random.default_rng(21)
    counts = rng.integers(0, 40000, 200).astype(np.int32)
    counts[:4] = [0, 1, 5, 102400]
    samples, offs, cnt = c.synth_reads(len(counts), counts, seed=42)
    host = samples.cpu().numpy()
    offs_h = offs.cpu().numpy()
    enc = c.compress_batch(samples, offs, cnt, with_stats=True)
    torch.cuda.synchronize()
    assert (enc.status.cpu().numpy() == 0).all()
    blobs = enc.blobs.cpu().numpy()
    bo, bs = enc.offsets.cpu().numpy(), enc.sizes.cpu().numpy()
    stats = enc.stats.cpu().numpy()
    for r in range(len(counts)):
        x = host[offs_h[r]:offs_h[r] + counts[r]]
        rc, ref, rst = O.variant_compress(variant, x)
        assert blobs[bo[r]:bo[r] + bs[r]].tobytes() == ref, (variant, r)
        assert np.array_equal(stats[r], rst.astype(np.int64)), (variant, r)
    out, so, dst = c.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cnt)
    torch.cuda.synchronize()
    assert (dst.cpu().numpy() == 0).all()
    assert torch.equal(out[: samples.numel()], samples[: out.numel()])


@pytest.mark.parametrize("variant", VARIANTS)
def test_errors_match_oracle(codecs, variant):
    from rawnanoporesignalcompression_amd import PGNanoError

    c = codecs[variant]
    x = np.random.default_rng(4).integers(-32768, 32768, 20000).astype(np.int16)
    rc, required, _ = O.variant_compress(variant, x)
    if rc != O.OK:
        with pytest.raises(PGNanoError) as ei:
            c.compress_signal(x)
        assert ei.value.status == rc
    y = O.synth_read(3, 20000)
    _, blob, _ = O.variant_compress(variant, y)
    cases = {
        "fewer": (blob, 19999), "more": (blob, 20001), "many_more": (blob, 30000), "zero": (blob, 0),
        "bad_magic": ((b"\0" + blob[1:]) if variant == "VBZ0" else (blob[:8] + b"\0" + blob[9:]), 20000),
        "truncated": (blob[:-5], 20000), "short": (blob[:6], 20000),
        "flipped": (blob[:70] + bytes([blob[70] ^ 0x5A]) + blob[71:], 20000),
    }
    for name, (b, n) in cases.items():
        orc, want = O.variant_decompress(variant, b, n)
        if orc == O.OK:
            assert np.array_equal(c.decompress_signal(b, sample_count=n), want), (variant, name)
        else:
            with pytest.raises(PGNanoError) as ei:
                c.decompress_signal(b, sample_count=n)
            assert ei.value.status == orc, (variant, name, ei.value.status, orc)


@pytest.mark.parametrize("variant", VARIANTS)
def test_decode_frames_from_other_encoder_settings(codecs, variant):
    """ZSTD_decompress takes any frame: blobs assembled from frames of other levels / windows."""
    c = codecs[variant]
    for level, wlog in [(3, 0), (19, 0), (1, 10), (22, 17)]:
        for i, n in enumerate([300, 20000, 102400]):
            x = O.synth_read(990 + i, n)
            frames = [O.zstd_compress_ex(s, level, wlog) for s in O.variant_streams(variant, x)]
            blob = frames[0] if variant == "VBZ0" else O.variant_assemble(frames)
            assert O.variant_decompress(variant, blob, n)[0] == O.OK
            assert np.array_equal(c.decompress_signal(blob, sample_count=n), x), (variant, level, wlog, n)
