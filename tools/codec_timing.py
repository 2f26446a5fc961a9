"""Encode/decode timing of R synthetic reads (default 20000 x 100000 samples), several repeats."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from rawnanoporesignalcompression_amd import PGNanoCodec

R = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
S = 100000
c = PGNanoCodec(0)
samples, offs, cnt = c.synth_reads(R, S, seed=42)
e, d = [], []
# PGN_TIMING_BOUND=1: the bounded batch calls (the chunk size known to the caller: no scan, intermediates
# spaced for it)
bound = {"max_chunk_samples": S} if os.environ.get("PGN_TIMING_BOUND") == "1" else {}
for _ in range(K + 1):
    enc = c.compress_batch(samples, offs, cnt, **bound)
    out, so, st = c.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cnt, **bound)
    torch.cuda.synchronize()
    e.append(c.last_encode_ms())
    d.append(c.last_decode_ms())
ok = bool(torch.equal(out, samples))
e, d = (sorted(e[1:]), sorted(d[1:])) if K > 0 else (e, d)
print(f"R={R} encode ms min {e[0]:.3f} med {e[len(e)//2]:.3f}  decode ms min {d[0]:.3f} med {d[len(d)//2]:.3f}  ok {ok}")
