"""Software-pipelined bench step experiment: the batch in two halves on two codec contexts, the
decode of half 1 overlapping the encode of half 2 (run via gpurun).  Prints the step time."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from rawnanoporesignalcompression_amd import PGNanoCodec

R = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
S = 100000
K = 3
c1, c2 = PGNanoCodec(0), PGNanoCodec(0)
samples, offs, cnt = c1.synth_reads(R, S, seed=42)
caps = torch.clamp(cnt.to(torch.int64) * 2 + 26, min=1024)
boffs = torch.zeros(R, dtype=torch.int64, device="cuda")
boffs[1:] = torch.cumsum(caps, 0)[:-1]
blobs = torch.empty(int(caps.sum().item()), dtype=torch.uint8, device="cuda")
dec = torch.empty_like(samples)
NP = int(os.environ.get("PARTS", "2"))
b = [R * i // NP for i in range(NP + 1)]
parts = [(slice(b[i], b[i + 1]), (c1, c2)[i % 2]) for i in range(NP)]


def serial():
    e = c1.compress_batch(samples, offs, cnt, out=blobs, out_offsets=boffs, out_caps=caps, stream=c1.stream)
    c1.decompress_batch(blobs, boffs, e.sizes, cnt, out=dec, out_offsets=offs, stream=c1.stream)


def pipelined():
    # part i: encode then decode on context i % 2; the decode of part i runs beside the encode of
    # part i + 1 (the other context's stream)
    for sl, c in parts:
        e = c.compress_batch(samples, offs[sl], cnt[sl], out=blobs, out_offsets=boffs[sl], out_caps=caps[sl],
                             stream=c.stream)
        c.decompress_batch(blobs, boffs[sl], e.sizes, cnt[sl], out=dec, out_offsets=offs[sl], stream=c.stream)


for name, fn in [("serial", serial), ("pipelined", pipelined)]:
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(K):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    ok = bool(torch.equal(dec, samples))
    dec.zero_()
    print(f"{name}: step ms {1e3 * min(t):.2f} (GS/s {R * S / min(t) / 1e9:.1f}) ok {ok}", flush=True)
