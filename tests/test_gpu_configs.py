"""GPU parity on the BASELINE.json configs the default bench does not run:

* configs[2] (GIAB 10.4.1 offline: the generator with R10.4.1 dwell) and the other pore chemistries
  -- full-size 100,000-sample chunks, sampled blobs byte-identical to the oracle, exact round trip,
  pgnano/VBZ size ratio below 1 (the ratio-parity claim of the --pgnano vs --VBZ comparison);
* configs[4] (mixed R9.4.1 / R10.3 / R10.4.1 corpus, decode only) -- oracle-produced blobs decoded
  by the batch decode kernels;
* one context driven from two HIP streams at once (encode on one, decode on the other): both
  results still equal the oracle's (the context orders its launches across streams).
"""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

# generator dwell per chemistry (p_switch in 1/65536 units; bench.py PORES)
PORES = {"r941": 7282, "r103": 6554, "r1041": 5243}


def _flat(blobs):
    sizes = np.array([len(b) for b in blobs], np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    return np.frombuffer(b"".join(blobs), np.uint8).copy(), offs, sizes


@pytest.mark.parametrize("pore", sorted(PORES))
def test_pore_configs_identical_and_ratio_below_vbz(codec, pore):
    import torch

    from rawnanoporesignalcompression_amd import VBZCodec

    n, k, pq = 100_000, 2048, PORES[pore]
    samples, offs, cnt = codec.synth_reads(k, n, seed=42, p_switch_q16=pq)
    enc = codec.compress_batch(samples, offs, cnt)
    out, _, dst = codec.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cnt)
    torch.cuda.synchronize()
    assert (enc.status == 0).all() and (dst == 0).all()
    assert torch.equal(out, samples)
    blobs = enc.blobs.cpu().numpy()
    bo, bs = enc.offsets.cpu().numpy(), enc.sizes.cpu().numpy()
    for r in list(range(0, k, 128)) + [k - 1]:
        x = O.synth_read(r, n, p_switch_q16=pq)
        rc, ref, _ = O.c5_compress(x)
        assert rc == 0 and blobs[bo[r]:bo[r] + bs[r]].tobytes() == ref, (pore, r)
    vz = VBZCodec(0)
    try:
        ev = vz.compress_batch(samples, offs, cnt)
        vout, _, vst = vz.decompress_batch(ev.blobs, ev.offsets, ev.sizes, cnt)
        torch.cuda.synchronize()
        assert (ev.status == 0).all() and (vst == 0).all()
        assert torch.equal(vout, samples)
        vb = ev.blobs.cpu().numpy()
        vo, vs = ev.offsets.cpu().numpy(), ev.sizes.cpu().numpy()
        for r in (0, k // 2, k - 1):
            assert vb[vo[r]:vo[r] + vs[r]].tobytes() == O.vbz_compress(O.synth_read(r, n, p_switch_q16=pq)), (pore, r)
        c5_bytes, vbz_bytes = int(enc.sizes.sum().item()), int(ev.sizes.sum().item())
    finally:
        vz.close()
    assert c5_bytes < vbz_bytes, (pore, c5_bytes, vbz_bytes)


def test_mixed_pore_decode_only(codec):
    """configs[4]: thirds of the corpus per chemistry, blobs made by the oracle, decoded in one batch."""
    import torch

    n, per = 100_000, 40
    xs, blobs = [], []
    for i, pq in enumerate(PORES.values()):
        for r in range(per):
            x = O.synth_read(1000 * i + r, n, p_switch_q16=pq)
            rc, b, _ = O.c5_compress(x)
            assert rc == 0
            xs.append(x)
            blobs.append(b)
    flat, offs, sizes = _flat(blobs)
    counts = np.full(len(xs), n, np.int32)
    dev = torch.device("cuda", 0)
    out, _, st = codec.decompress_batch(torch.from_numpy(flat).to(dev), torch.from_numpy(offs).to(dev),
                                        torch.from_numpy(sizes).to(dev), torch.from_numpy(counts).to(dev))
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert np.array_equal(out.cpu().numpy(), np.concatenate(xs))


def test_one_context_two_streams(codec):
    """An encode on stream A and a decode on stream B of the same context, issued through the C ABI
    back to back with no host synchronisation and no stream dependency between them: the context's
    work counters and slot scratch are shared, so the library itself must order the calls on the
    device; both results equal the oracle's."""
    import torch

    n, k = 100_000, 1024
    dev = torch.device("cuda", 0)
    lib, h = codec._lib, codec._h
    # batch B: blobs made up front by the oracle, decoded on stream B
    xb, bb = [], []
    for r in range(64):
        x = O.synth_read(5000 + r, n)
        xb.append(x)
        bb.append(O.c5_compress(x)[1])
    flat, offs_b, sizes_b = _flat(bb)
    d_flat, d_ob, d_sb = (torch.from_numpy(a).to(dev) for a in (flat, offs_b, sizes_b))
    d_cb = torch.full((len(xb),), n, dtype=torch.int32, device=dev)
    d_so = torch.arange(len(xb), dtype=torch.int64, device=dev) * n
    # batch A: device samples, encoded on stream A (two output sets)
    samples, offs, cnt = codec.synth_reads(k, n, seed=42)
    caps = torch.clamp(cnt.to(torch.int64) * 2 + 26, min=1024)
    bo = torch.zeros(k, dtype=torch.int64, device=dev)
    bo[1:] = torch.cumsum(caps, 0)[:-1]
    outs = [torch.empty(int(caps.sum().item()), dtype=torch.uint8, device=dev) for _ in range(2)]
    sizes = [torch.zeros(k, dtype=torch.int64, device=dev) for _ in range(2)]
    stats = [torch.full((k,), -1, dtype=torch.int32, device=dev) for _ in range(2)]
    dec = torch.empty(len(xb) * n, dtype=torch.int16, device=dev)
    dst = torch.full((len(xb),), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for _ in range(2):
        for i, s in enumerate((sa, sb)):
            assert lib.pgn_compress_batch_device(h, k, samples.data_ptr(), offs.data_ptr(), cnt.data_ptr(),
                                                 outs[i].data_ptr(), bo.data_ptr(), caps.data_ptr(),
                                                 sizes[i].data_ptr(), stats[i].data_ptr(), None, s.cuda_stream) == 0
            assert lib.pgn_decompress_batch_device(h, len(xb), d_flat.data_ptr(), d_ob.data_ptr(), d_sb.data_ptr(),
                                                   dec.data_ptr(), d_so.data_ptr(), d_cb.data_ptr(), dst.data_ptr(),
                                                   (sb if i == 0 else sa).cuda_stream) == 0
    torch.cuda.synchronize()
    assert (stats[0] == 0).all() and (stats[1] == 0).all() and (dst == 0).all()
    assert np.array_equal(dec.cpu().numpy(), np.concatenate(xb))
    assert torch.equal(sizes[0], sizes[1])
    b0, b1 = outs[0].cpu().numpy(), outs[1].cpu().numpy()
    bo_h, bs_h = bo.cpu().numpy(), sizes[0].cpu().numpy()
    assert np.array_equal(b0, b1) or all(
        b0[bo_h[r]:bo_h[r] + bs_h[r]].tobytes() == b1[bo_h[r]:bo_h[r] + bs_h[r]].tobytes() for r in range(k))
    for r in list(range(0, k, 61)) + [k - 1]:
        ref = O.c5_compress(O.synth_read(r, n))[1]
        assert b0[bo_h[r]:bo_h[r] + bs_h[r]].tobytes() == ref, r


def _deferred_codec(min_chunks: str, group: str):
    import os

    from rawnanoporesignalcompression_amd import PGNanoCodec

    keys = ("PGN_DEFER_MIN_CHUNKS", "PGN_DEFER_G")
    old = {k: os.environ.get(k) for k in keys}
    os.environ["PGN_DEFER_MIN_CHUNKS"], os.environ["PGN_DEFER_G"] = min_chunks, group
    try:
        return PGNanoCodec(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_mixed_pore_decode_only_deferred_path():
    """configs[4]'s corpus through the production decode path of large batches (the deferred
    four-stream Huffman sections, dec_huf_kernel) in passes of 48 chunks (both pass buffers, three
    passes): oracle-made blobs of every chemistry, samples equal to the oracle's reads."""
    import torch

    n, per = 100_000, 40
    xs, blobs = [], []
    for i, pq in enumerate(PORES.values()):
        for r in range(per):
            x = O.synth_read(1000 * i + r, n, p_switch_q16=pq)
            rc, b, _ = O.c5_compress(x)
            assert rc == 0
            xs.append(x)
            blobs.append(b)
    flat, offs, sizes = _flat(blobs)
    counts = np.full(len(xs), n, np.int32)
    dev = torch.device("cuda", 0)
    c = _deferred_codec("1", "48")
    try:
        out, _, st = c.decompress_batch(torch.from_numpy(flat).to(dev), torch.from_numpy(offs).to(dev),
                                        torch.from_numpy(sizes).to(dev), torch.from_numpy(counts).to(dev))
        torch.cuda.synchronize()
        assert "dec_huf_kernel" in c.kernels(1)
    finally:
        c.close()
    assert (st.cpu().numpy() == 0).all()
    assert np.array_equal(out.cpu().numpy(), np.concatenate(xs))


def test_mixed_pore_decode_at_production_defaults(codec):
    """configs[4] at the default thresholds: 12,600 mixed-chemistry chunks (above PGN_DEFER_MIN_CHUNKS
    = 12,288, so the deferred path the configs[4] bench line runs), encoded on the GPU (sampled blobs
    equal to the oracle's) and decoded back exactly."""
    import torch

    n, k = 100_000, 12600
    dev = torch.device("cuda", 0)
    samples = torch.empty(k * n, dtype=torch.int16, device=dev)
    cuts = [0, k // 3, 2 * k // 3, k]
    pqs = list(PORES.values())
    for i, pq in enumerate(pqs):
        a, e = cuts[i], cuts[i + 1]
        codec.synth_reads(e - a, n, seed=42, first_read=a, p_switch_q16=pq, out=samples[a * n:e * n])
    offs = torch.arange(k, dtype=torch.int64, device=dev) * n
    cnt = torch.full((k,), n, dtype=torch.int32, device=dev)
    enc = codec.compress_batch(samples, offs, cnt)
    out, _, st = codec.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cnt)
    torch.cuda.synchronize()
    assert "dec_huf_kernel" in codec.kernels(1)
    assert (enc.status == 0).all() and (st == 0).all()
    assert torch.equal(out, samples)
    blobs, bo, bs = enc.blobs, enc.offsets.cpu().numpy(), enc.sizes.cpu().numpy()
    for r in (0, 1, k // 3 - 1, k // 3, 2 * k // 3 + 7, k - 1):
        i = 0 if r < cuts[1] else (1 if r < cuts[2] else 2)
        x = O.synth_read(r, n, p_switch_q16=pqs[i])
        assert np.array_equal(samples[r * n:(r + 1) * n].cpu().numpy(), x), r
        rc, ref, _ = O.c5_compress(x)
        assert rc == 0 and blobs[bo[r]:bo[r] + bs[r]].cpu().numpy().tobytes() == ref, r
