"""Small-batch kernels under contention: context A's 64-chunk calls (the look-back split / merge,
the cooperative stream encode whose frames place themselves, the cooperative frame decode -- kernels
whose workgroups wait on lower-numbered workgroups of the same launch) issued while context B's long
batch encodes hold the CUs on another stream.  A workgroup only ever waits on lower-numbered ones,
which the dispatcher started first, so A's kernels finish whatever share of the chip B leaves them;
A's blobs and samples must equal the oracle's (C5.hpp:429-462 frame order, :173-257 merge)."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


def test_small_batches_beside_a_long_batch_encode():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rawnanoporesignalcompression_amd import PGNanoCodec

    dev = torch.device("cuda", 0)
    A, B = PGNanoCodec(0), PGNanoCodec(0)
    try:
        # B: 24,000 full-size reads, encoded four times back to back (~20 ms of chip time); its
        # output buffers are given, so no call waits on the host
        nb, n = 24000, 100000
        sB, oB, cB = B.synth_reads(nb, n, seed=5)
        capsB = torch.full((nb,), 2 * n + 26, dtype=torch.int64, device=dev)
        ooB = torch.arange(nb, dtype=torch.int64, device=dev) * (2 * n + 26)
        outB = torch.empty(nb * (2 * n + 26), dtype=torch.uint8, device=dev)
        # A: 64 chunks of varied sizes (per-chunk-path kernels: at most 64 chunks per call)
        xs = [O.synth_read(600 + i, 100000 - 997 * i) for i in range(64)]
        ref = [O.c5_compress(x) for x in xs]
        assert all(r[0] == 0 for r in ref)
        cnt = np.array([x.size for x in xs], np.int32)
        offs = np.concatenate([[0], np.cumsum(cnt[:-1].astype(np.int64))])
        sA = torch.from_numpy(np.concatenate(xs)).to(dev)
        oA, cA = torch.from_numpy(offs).to(dev), torch.from_numpy(cnt).to(dev)
        torch.cuda.synchronize()

        tB, tA = torch.cuda.Stream(), torch.cuda.Stream()
        t0 = torch.cuda.Event(enable_timing=True)
        eB, eA = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(tB)
        tA.wait_event(t0)
        with torch.cuda.stream(tB):
            for _ in range(4):
                encB = B.compress_batch(sB, oB, cB, out=outB, out_offsets=ooB, out_caps=capsB)
            eB.record(tB)
        rounds = []
        with torch.cuda.stream(tA):
            for _ in range(6):
                enc = A.compress_batch(sA, oA, cA)
                dec, _, st = A.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cA)
                rounds.append((enc, dec, st))
            eA.record(tA)
        torch.cuda.synchronize()
        print(f"A's six rounds ended {t0.elapsed_time(eA):.2f} ms after B started; B's encodes "
              f"{t0.elapsed_time(eB):.2f} ms")
        for enc, dec, st in rounds:
            assert (enc.status.cpu().numpy() == 0).all()
            sizes, blobs, boffs = enc.sizes.cpu().numpy(), enc.blobs.cpu().numpy(), enc.offsets.cpu().numpy()
            for i, (rc, b, _) in enumerate(ref):
                assert bytes(blobs[boffs[i]:boffs[i] + sizes[i]]) == b, i
            assert (st.cpu().numpy() == 0).all()
            assert torch.equal(dec, sA)
        assert (encB.status == 0).all()
    finally:
        A.close()
        B.close()
