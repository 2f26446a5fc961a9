"""GPU tests of the batched POD5 signal-table integration (include/pgnano_pod5.h): the C program
linked against the header, the reference fixture's signal column reproduced by one batched call, and
pgnano batches equal to the per-chunk oracle.  Needs an MI355X."""
import os
import subprocess

import numpy as np
import pytest

import _oracle as O
from _golden import real_vbz_chunks

def _have_gpu():
    import torch

    return torch.cuda.is_available()


pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not _have_gpu(), reason="no GPU")]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_program():
    exe = os.path.join(ROOT, "rawnanoporesignalcompression_amd", "_build", "test_pod5_batch")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "pod5 batch: ok" in r.stdout


def _fixture_reads():
    """The fixture's reads: its signal rows grouped back into reads (a read's rows are consecutive,
    all but its last exactly the writer's 102,400-sample chunk)."""
    reads, cur = [], []
    for blob, n in real_vbz_chunks():
        rc, x = O.vbz_decompress(blob, n)
        assert rc == 0
        cur.append(x)
        if n < 102400:
            reads.append(np.concatenate(cur))
            cur = []
    assert not cur
    return reads


def test_reference_signal_column_reproduced():
    """pod5_add_reads_data of the fixture's 10 reads with --VBZ: the batched call returns exactly the
    signal column the reference writer wrote (row sizes, samples and bytes)."""
    from rawnanoporesignalcompression_amd import Pod5SignalBatch, VBZCodec

    reads = _fixture_reads()
    assert len(reads) == 10
    want = real_vbz_chunks()
    vz = VBZCodec(0)
    b = Pod5SignalBatch(vz)
    try:
        offsets, data, samples, read_index = b.compress_reads(reads)
        assert len(samples) == len(want)
        for i, (blob, n) in enumerate(want):
            assert samples[i] == n and data[offsets[i]:offsets[i + 1]].tobytes() == blob, i
        assert np.array_equal(b.decompress_rows(offsets, data, samples), np.concatenate(reads))
    finally:
        b.close()
        vz.close()


@pytest.mark.parametrize("chunk", [0, 65536, 262144, 1048576])
def test_pgnano_batch_matches_per_chunk_oracle(codec, chunk):
    from rawnanoporesignalcompression_amd import Pod5SignalBatch

    rng = np.random.default_rng(chunk + 1)
    lens = rng.integers(0, 400000, 60)
    lens[:3] = [0, 1, 102400]
    reads = [O.synth_read(100 + i, int(n)) for i, n in enumerate(lens)]
    b = Pod5SignalBatch(codec, chunk)
    try:
        offsets, data, samples, read_index = b.compress_reads(reads)
        cs = chunk or 102400
        i = 0
        for r, x in enumerate(reads):
            for s in range(0, x.size, cs):
                piece = x[s:s + cs]
                assert read_index[i] == r and samples[i] == piece.size
                if i % 5 == 0:
                    rc, ref, _ = O.c5_compress(piece)
                    assert rc == 0 and data[offsets[i]:offsets[i + 1]].tobytes() == ref, (r, s)
                i += 1
        assert i == len(samples)
        assert np.array_equal(b.decompress_rows(offsets, data, samples), np.concatenate(reads))
    finally:
        b.close()


def test_uniform_noise_chunks_fail_without_fault(codec):
    """Chunks the codec refuses (uniform noise does not fit pgnano's 2n + 26 bound, compressor.h:39-45)
    fail the call with PGN_ERR_DST_TOO_SMALL at the first failing chunk; the packing scan skips
    failed chunks' sizes, so nothing is written out of bounds, and the batch keeps working."""
    from rawnanoporesignalcompression_amd import PGNanoError, Pod5SignalBatch

    rng = np.random.default_rng(7)
    good = [O.synth_read(900 + i, 150000) for i in range(6)]
    noise = [rng.integers(-32768, 32767, 102400 * 3, dtype=np.int16) for _ in range(40)]
    b = Pod5SignalBatch(codec)
    try:
        with pytest.raises(PGNanoError) as e:
            b.compress_reads(good + noise)
        assert e.value.status == 1  # PGN_ERR_DST_TOO_SMALL
        assert "chunk 12" in str(e.value)  # 6 good reads x 2 chunks, then the first noise chunk
        offsets, data, samples, _ = b.compress_reads(good)
        assert len(samples) == 12
        for i in (0, 5, 11):
            rc, ref, _ = O.c5_compress(good[i // 2][(i % 2) * 102400:(i % 2 + 1) * 102400])
            assert rc == 0 and data[offsets[i]:offsets[i + 1]].tobytes() == ref
    finally:
        b.close()
