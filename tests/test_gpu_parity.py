"""GPU parity: the gfx950 codec, called through the C ABI, against the oracle (libzstd-backed C
restatement of C5.hpp) -- byte-identical blobs and bit-exact samples.  Needs an MI355X."""
import hashlib

import numpy as np
import pytest

import _oracle as O
from _golden import c5_blobs, golden, real_vbz_chunks

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_real_pod5_chunks_identical(codec):
    """Every chunk of the reference's POD5 fixture: same C5 bytes as the oracle, exact round trip."""
    g = golden()["real"]
    tot_c5 = tot_n = 0
    for (vbz, n), meta in zip(real_vbz_chunks(), g):
        rc, x = O.vbz_decompress(vbz, n)
        assert rc == 0
        blob = codec.compress_signal(x)
        assert len(blob) == meta["c5_size"]
        assert sha(blob) == meta["c5_sha256"], f"chunk {meta['chunk']}"
        back = codec.decompress_signal(blob, sample_count=n)
        assert np.array_equal(back, x)
        tot_c5 += len(blob)
        tot_n += n
    assert abs(8.0 * tot_c5 / tot_n - golden()["real_totals"]["c5_bits_per_sample"]) < 1e-12


def test_decode_committed_blobs(codec):
    for name, blob in c5_blobs().items():
        if name.startswith("real"):
            i = int(name[4:])
            vbz, n = real_vbz_chunks()[i]
            _, want = O.vbz_decompress(vbz, n)
        else:
            want = O.synth_read(7, 3000)
        got = codec.decompress_signal(blob, sample_count=want.size)
        assert np.array_equal(got, want)


def test_edge_sizes_identical(codec):
    for e in golden()["edge"]:
        n = e["samples"]
        x = O.synth_read(1000 + n, n)
        blob = codec.compress_signal(x)
        assert sha(blob) == e["c5_sha256"], n
        assert np.array_equal(codec.decompress_signal(blob, sample_count=n), x)


def _pattern_signals():
    rng = np.random.default_rng(5)
    sig = {}
    sig["constant"] = np.full(50000, 417, np.int16)
    sig["alternating_extremes"] = np.tile(np.array([32767, -32768], np.int16), 20000)
    sig["ramp"] = (np.arange(70000) % 65536 - 32768).astype(np.int16)
    base = rng.integers(400, 600, 257).astype(np.int16)
    sig["periodic257"] = np.tile(base, 300)
    sig["periodic_noisy"] = (np.tile(base, 300) + (rng.random(257 * 300) < 0.01) * 40).astype(np.int16)
    steps = np.repeat(rng.integers(300, 700, 2000), rng.integers(1, 60, 2000))[:90000]
    sig["steps_no_noise"] = steps.astype(np.int16)
    sig["small_uniform"] = rng.integers(-32768, 32768, 300).astype(np.int16)
    sig["spiky"] = np.where(rng.random(60000) < 0.02, rng.integers(-30000, 30000, 60000),
                            500 + rng.integers(-3, 4, 60000)).astype(np.int16)
    sig["bimodal_deltas"] = np.cumsum(rng.choice([-300, 0, 1, 300], 80000)).astype(np.int16)
    return sig


def test_pattern_signals_identical(codec):
    """Signals whose streams carry zstd sequences (repeats), RLE literals, raw and 4-stream Huffman."""
    for name, x in _pattern_signals().items():
        rc, ref, _ = O.c5_compress(x)
        assert rc == 0, name
        blob = codec.compress_signal(x)
        assert blob == ref, name
        assert np.array_equal(codec.decompress_signal(ref, sample_count=x.size), x), name


def test_not_enough_space_matches_reference(codec):
    """Uniform int16 does not fit max(2n+26,1024): the reference returns Invalid (C5.hpp:420-427)."""
    from rawnanoporesignalcompression_amd import PGNanoError

    x = np.random.default_rng(1).integers(-32768, 32768, 100000).astype(np.int16)
    rc, required, _ = O.c5_compress(x)
    assert rc == O.DST_TOO_SMALL
    with pytest.raises(PGNanoError, match="Not enough space in destination buffer") as ei:
        codec.compress_signal(x)
    assert f"Required size: {required}" in str(ei.value)


def test_decode_error_statuses_match_oracle(codec):
    from rawnanoporesignalcompression_amd import PGNanoError

    x = O.synth_read(3, 20000)
    rc, blob, _ = O.c5_compress(x)
    cases = {
        "wrong_count": (blob, 19999),
        "bad_magic": (blob[:8] + b"\x00" + blob[9:], 20000),
        "truncated": (blob[:-5], 20000),
        "short": (blob[:12], 20000),
        "flipped_payload": (blob[:60] + bytes([blob[60] ^ 0x5A]) + blob[61:], 20000),
    }
    for name, (b, n) in cases.items():
        orc, _ = O.c5_decompress(b, n)
        if orc == 0:
            got = codec.decompress_signal(b, sample_count=n)
            assert np.array_equal(got, O.c5_decompress(b, n)[1]), name
        else:
            with pytest.raises(PGNanoError) as ei:
                codec.decompress_signal(b, sample_count=n)
            assert ei.value.status == orc, (name, ei.value.status, orc)


def test_batch_device_identical_and_round_trip(codec):
    import torch

    rng = np.random.default_rng(11)
    counts = rng.integers(0, 40000, 300).astype(np.int32)
    counts[:4] = [0, 1, 5, 102400]
    samples, offs, cnt = codec.synth_reads(len(counts), counts, seed=42)
    host = samples.cpu().numpy()
    offs_h = offs.cpu().numpy()
    for r in range(len(counts)):  # the device generator is the checker's generator
        assert np.array_equal(host[offs_h[r]:offs_h[r] + counts[r]], O.synth_read(r, int(counts[r]))), r
    enc = codec.compress_batch(samples, offs, cnt, with_stats=True)
    torch.cuda.synchronize()
    st = enc.status.cpu().numpy()
    assert (st == 0).all(), np.unique(st)
    blobs = enc.blobs.cpu().numpy()
    bo, bs = enc.offsets.cpu().numpy(), enc.sizes.cpu().numpy()
    stats = enc.stats.cpu().numpy()
    for r in range(len(counts)):
        x = host[offs_h[r]:offs_h[r] + counts[r]]
        rc, ref, rst = O.c5_compress(x)
        got = blobs[bo[r]:bo[r] + bs[r]].tobytes()
        assert got == ref, r
        assert np.array_equal(stats[r], rst.astype(np.int64)), r
    out, so, dst = codec.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cnt)
    torch.cuda.synchronize()
    assert (dst.cpu().numpy() == 0).all()
    assert torch.equal(out[: samples.numel()], samples[: out.numel()])


@pytest.mark.slow
def test_full_size_chunks_round_trip(codec):
    """BASELINE config sizes (100,000-sample chunks): round trip of 4096 chunks on device, every
    blob's size/hash equal to the oracle's on a sampled subset."""
    import torch

    n, k = 100000, 4096
    samples, offs, cnt = codec.synth_reads(k, n, seed=42)
    enc = codec.compress_batch(samples, offs, cnt)
    out, so, dst = codec.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cnt)
    torch.cuda.synchronize()
    assert (enc.status == 0).all() and (dst == 0).all()
    assert torch.equal(out, samples)
    blobs = enc.blobs.cpu().numpy()
    bo, bs = enc.offsets.cpu().numpy(), enc.sizes.cpu().numpy()
    for r in list(range(0, k, 97)) + [k - 1]:
        rc, ref, _ = O.c5_compress(O.synth_read(r, n))
        assert blobs[bo[r]:bo[r] + bs[r]].tobytes() == ref, r
    bits = 8.0 * float(enc.sizes.sum().item()) / (n * k)
    assert 5.0 < bits < 8.0


def test_decode_frames_from_other_encoder_settings(codec):
    """The reference decodes whatever libzstd frames a blob holds (ZSTD_decompress, C5.hpp:520-600).
    Blobs whose five frames come from other levels (compressed FSE sequence tables, 1-stream
    literals, long matches) or forced small windows (multi-block frames, repeat-mode tables,
    window-descriptor headers) decode to the original samples -- one at a time and batched."""
    import torch

    settings = [(3, 0), (9, 0), (19, 0), (-5, 0), (1, 10), (6, 12), (19, 11), (22, 17)]
    sigs = [O.synth_read(900 + i, n) for i, n in enumerate([5, 300, 4099, 20000, 65792, 102400, 131072])]
    sigs += list(_pattern_signals().values())
    blobs, want = [], []
    for level, wlog in settings:
        for x in sigs:
            blob = O.c5_assemble([O.zstd_compress_ex(s, level, wlog) for s in O.c5_streams(x)])
            got = codec.decompress_signal(blob, sample_count=x.size)
            assert np.array_equal(got, x), (level, wlog, x.size)
            blobs.append(blob)
            want.append(x)
    sizes = np.array([len(b) for b in blobs], np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    flat = np.frombuffer(b"".join(blobs), np.uint8)
    counts = np.array([w.size for w in want], np.int32)
    dev = torch.device("cuda", 0)
    out, so, st = codec.decompress_batch(torch.from_numpy(flat.copy()).to(dev), torch.from_numpy(offs).to(dev),
                                         torch.from_numpy(sizes).to(dev), torch.from_numpy(counts).to(dev))
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert np.array_equal(out.cpu().numpy()[: counts.sum()], np.concatenate(want))


def _huffman_stress_signals():
    """Delta distributions from very skewed (1-2 bit Huffman codes, hundreds of symbols per lane
    window) to wide (11-bit codes): every shape the speculative Huffman rounds must resynchronise on."""
    rng = np.random.default_rng(11)
    sig = {}
    for p in (0.97, 0.9, 0.6, 0.3, 0.1, 0.03):
        d = rng.geometric(p, 131072) - 1
        d = np.where(rng.random(d.size) < 0.5, d, -d)
        sig[f"geometric_p{p}"] = np.cumsum(d).astype(np.int16)
    for sd in (1, 40, 3000):
        sig[f"gauss_sd{sd}"] = (np.cumsum(rng.normal(0, sd, 102400)).round() % 65536 - 32768).astype(np.int16)
    sig["mostly_zero_deltas"] = np.cumsum((rng.random(102400) < 0.002) * rng.integers(-9, 10, 102400)).astype(np.int16)
    return sig


@pytest.mark.gpu
def test_huffman_stress_signals_identical(codec):
    """Encoder bytes = oracle bytes, and the GPU decoder round-trips the oracle's blob, one at a time
    and batched (the batched path runs the staged decode kernels)."""
    import torch

    sigs = list(_huffman_stress_signals().items())
    blobs = []
    for name, x in sigs:
        rc, ref, _ = O.c5_compress(x)
        if rc != 0:  # wider than max(2n+26, 1024): the reference refuses it as well
            continue
        assert codec.compress_signal(x) == ref, name
        assert np.array_equal(codec.decompress_signal(ref, sample_count=x.size), x), name
        blobs.append((ref, x))
    assert len(blobs) >= 8
    sizes = np.array([len(b) for b, _ in blobs], np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    flat = np.frombuffer(b"".join(b for b, _ in blobs), np.uint8)
    counts = np.array([x.size for _, x in blobs], np.int32)
    dev = torch.device("cuda", 0)
    out, so, st = codec.decompress_batch(torch.from_numpy(flat.copy()).to(dev), torch.from_numpy(offs).to(dev),
                                         torch.from_numpy(sizes).to(dev), torch.from_numpy(counts).to(dev))
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert np.array_equal(out.cpu().numpy()[: counts.sum()], np.concatenate([x for _, x in blobs]))


def test_small_batches_take_the_workgroup_split_and_merge(codec):
    """Batches of up to 64 chunks split and merge each chunk with a 16-wave workgroup (range class
    counts, shared S bytes at odd nibble starts, order-free delta sums); larger batches with one wave
    per chunk.  Both give the oracle's blobs and the same samples and statuses, corrupted blobs
    included."""
    import torch

    rng = np.random.default_rng(64)
    lens = rng.integers(0, 262145, 65).astype(np.int32)
    lens[:6] = [0, 1, 1023, 1024, 1025, 16 * 1024 + 7]
    reads = [O.synth_read(5000 + i, int(n)) if i % 3 else
             np.clip(rng.normal(0, 10 + 20 * (i % 5), int(n)), -32768, 32767).astype(np.int16)
             for i, n in enumerate(lens)]
    flat = np.concatenate(reads)
    dev = torch.device("cuda", 0)
    samples = torch.from_numpy(flat).to(dev)
    counts = torch.from_numpy(lens).to(dev)
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(lens.astype(np.int64))[:-1]])).to(dev)
    whole = codec.compress_batch(samples, offs, counts)          # 65 chunks: one wave per chunk
    parts = [codec.compress_batch(samples, offs[a:b], counts[a:b]) for a, b in ((0, 33), (33, 65))]
    torch.cuda.synchronize()
    wb, wo, ws = whole.blobs.cpu().numpy(), whole.offsets.cpu().numpy(), whole.sizes.cpu().numpy()
    blobs = []
    for (a, b), p in zip(((0, 33), (33, 65)), parts):
        pb, po, ps = p.blobs.cpu().numpy(), p.offsets.cpu().numpy(), p.sizes.cpu().numpy()
        for i in range(b - a):
            blob = pb[po[i]:po[i] + ps[i]].tobytes()
            assert blob == wb[wo[a + i]:wo[a + i] + ws[a + i]].tobytes(), a + i
            blobs.append(blob)
    for i in list(range(0, 65, 4)) + [1, 2, 3, 4, 5]:
        rc, ref, _ = O.c5_compress(reads[i])
        assert rc == 0 and blobs[i] == ref, i
    # decode: valid and corrupted blobs, one batch of 65 vs two of <= 64
    bad = [bytearray(b) for b in blobs]
    for i in range(0, 65, 5):
        if len(bad[i]) > 40:
            bad[i][len(bad[i]) // 2] ^= 0x5A
    for i in range(2, 65, 7):
        bad[i] = bad[i][:-3] if len(bad[i]) > 50 else bad[i]
    data = b"".join(bytes(b) for b in bad)
    bsz = np.array([len(b) for b in bad], np.int64)
    boff = np.concatenate([[0], np.cumsum(bsz)[:-1]]).astype(np.int64)
    din = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(dev)
    ob, sb = torch.from_numpy(boff).to(dev), torch.from_numpy(bsz).to(dev)
    out_w, _, st_w = codec.decompress_batch(din, ob, sb, counts)
    res = [codec.decompress_batch(din, ob[a:b], sb[a:b], counts[a:b]) for a, b in ((0, 33), (33, 65))]
    torch.cuda.synchronize()
    st_p = torch.cat([r[2] for r in res]).cpu().numpy()
    assert np.array_equal(st_w.cpu().numpy(), st_p)
    ow = out_w.cpu().numpy()
    so = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    for k, (a, b) in enumerate(((0, 33), (33, 65))):
        op = res[k][0].cpu().numpy()
        base = so[a]
        for i in range(a, b):
            rc, ref = O.c5_decompress(bytes(bad[i]), int(lens[i]))
            if rc == 0 and st_p[i] == 3 and not O.c5_frames_strictly_valid(bytes(bad[i])):
                continue  # libzstd's double-symbol decoder accepts one trailing codeword
            assert st_p[i] == rc, (i, rc, st_p[i])
            if rc == 0:
                assert np.array_equal(op[so[i] - base:so[i + 1] - base], ref), i
                assert np.array_equal(ow[so[i]:so[i + 1]], ref), i
