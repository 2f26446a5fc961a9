"""Diagnostic: encode + decode a few synthetic reads and print the per-stream decode records."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch

from rawnanoporesignalcompression_amd import PGNanoCodec

R = int(sys.argv[1]) if len(sys.argv) > 1 else 6
S = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
c = PGNanoCodec(0)
samples, offs, cnt = c.synth_reads(R, S, seed=42)
enc = c.compress_batch(samples, offs, cnt, with_stats=True)
dec, _, st = c.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cnt)
torch.cuda.synchronize()
print("enc status", enc.status.cpu().tolist())
print("dec status", st.cpu().tolist())
rec = np.zeros(R * 5 * 3, dtype=np.uint64)
c._lib.pgn_debug_decode_units(c._h, rec.ctypes.data, R)
raw = rec.view(np.uint32).reshape(R, 5, 6)
stats = enc.stats.cpu().numpy()
for i in range(min(R, 3)):
    print(i, "raw", stats[i, :5].tolist(), "frames", stats[i, 5:].tolist())
    print("   dec (len, cs, res):", [(int(r[2]), int(r[3]), int(np.int32(r[5]))) for r in raw[i]])
ok = torch.equal(dec, samples)
print("round trip", ok)
if not ok:
    d = (dec != samples).nonzero()
    print("first mismatch at", d[:5].flatten().tolist())
stt = st.cpu().numpy()
bad = np.nonzero(stt != 0)[0]
print("failed chunks", len(bad), "of", R)
codes = {}
for i in bad[:2000]:
    for sidx, r in enumerate(raw[i]):
        v = int(np.int32(r[5]))
        if v < 0:
            codes[(sidx, v)] = codes.get((sidx, v), 0) + 1
print("failure (stream, code) counts:", codes)
