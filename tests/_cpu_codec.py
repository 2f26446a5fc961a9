"""CPU stand-in for PGNanoCodec with the same batch methods, backed by the oracle -- test
infrastructure only: it lets tests/test_dist.py drive bench.py's own rank body (bench.run_rank)
under gloo on CPU, so the orchestration (partition, batches, barriers, reduction, the bench line) is
tested without a GPU.  Never used by the product path or by bench.py itself."""
import time
from types import SimpleNamespace

import numpy as np
import torch

import _oracle as O


class CpuCodec:
    stream = 0

    def __init__(self):
        self._enc_ms = self._dec_ms = 0.0

    def synth_reads(self, nreads, S, seed=42, first_read=0, read_stride=1, p_switch_q16=6554, out=None):
        for r in range(nreads):
            x = O.synth_read(first_read + r * read_stride, S, seed=seed, p_switch_q16=p_switch_q16)
            out[r * S:(r + 1) * S] = torch.from_numpy(x)
        return out, torch.arange(nreads, dtype=torch.int64) * S, torch.full((nreads,), S, dtype=torch.int32)

    def compress_batch(self, samples, offs, counts, out=None, out_offsets=None, out_caps=None, stream=None):
        t0 = time.perf_counter()
        n = counts.numel()
        sizes = torch.zeros(n, dtype=torch.int64)
        status = torch.zeros(n, dtype=torch.int32)
        ob = out.numpy()
        for i in range(n):
            o, c = int(offs[i]), int(counts[i])
            rc, blob, _ = O.c5_compress(samples[o:o + c].numpy(), int(out_caps[i]))
            status[i] = rc
            if rc == 0:
                oo = int(out_offsets[i])
                ob[oo:oo + len(blob)] = np.frombuffer(blob, np.uint8)
                sizes[i] = len(blob)
        self._enc_ms = 1e3 * (time.perf_counter() - t0)
        return SimpleNamespace(blobs=out, offsets=out_offsets, caps=out_caps, sizes=sizes, status=status)

    def decompress_batch(self, blobs, boffs, sizes, counts, out=None, out_offsets=None, stream=None):
        t0 = time.perf_counter()
        b = blobs.numpy()
        n = counts.numel()
        status = torch.zeros(n, dtype=torch.int32)
        for i in range(n):
            bo, bs, c, so = int(boffs[i]), int(sizes[i]), int(counts[i]), int(out_offsets[i])
            rc, x = O.c5_decompress(b[bo:bo + bs].tobytes(), c)
            status[i] = rc
            if rc == 0:
                out[so:so + c] = torch.from_numpy(x)
        self._dec_ms = 1e3 * (time.perf_counter() - t0)
        return out, out_offsets, status

    def last_encode_ms(self):
        return self._enc_ms

    def last_decode_ms(self):
        return self._dec_ms

    def kernels(self, direction):
        return "cpu stand-in (oracle)"
