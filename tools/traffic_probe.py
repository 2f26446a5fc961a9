"""One bench step (encode + decode of R reads x S samples, the bench's buffers and launch sequence)
for the HBM-traffic passes of tools/traffic.sh.  Run under rocprofv3 --pmc on the GPU box.
A third argument "mixed" generates configs[4]'s corpus (thirds with the R9.4.1 / R10.3 / R10.4.1
generator dwell, bench.py --mixed-pores); its decode is the measured direction there."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from rawnanoporesignalcompression_amd import PGNanoCodec

R = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
S = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
c = PGNanoCodec(0)
samples = torch.empty(R * S, dtype=torch.int16, device="cuda")
counts = torch.full((R,), S, dtype=torch.int32, device="cuda")
offs = torch.arange(R, dtype=torch.int64, device="cuda") * S
if len(sys.argv) > 3 and sys.argv[3] == "mixed":  # bench.py PORES, thirds of the batch
    cuts = [0, R // 3, 2 * R // 3, R]
    for i, pq in enumerate((7282, 6554, 5243)):
        a, e = cuts[i], cuts[i + 1]
        c.synth_reads(e - a, S, seed=42, first_read=a, p_switch_q16=pq, out=samples[a * S:e * S])
else:
    c.synth_reads(R, S, seed=42, out=samples)
caps = torch.clamp(counts.to(torch.int64) * 2 + 26, min=1024)
boffs = torch.zeros(R, dtype=torch.int64, device="cuda")
boffs[1:] = torch.cumsum(caps, 0)[:-1]
blobs = torch.empty(int(caps.sum().item()), dtype=torch.uint8, device="cuda")
decoded = torch.empty(R * S, dtype=torch.int16, device="cuda")
torch.cuda.synchronize()
enc = c.compress_batch(samples, offs, counts, out=blobs, out_offsets=boffs, out_caps=caps, stream=c.stream)
if os.environ.get("PGN_ENCODE_ONLY") != "1":  # (the diagnostic encode builds' blobs are not decodable)
    c.decompress_batch(blobs, boffs, enc.sizes, counts, out=decoded, out_offsets=offs, stream=c.stream)
torch.cuda.synchronize()
comp = int(enc.sizes.sum().item())
print(f"reads {R} samples {S} compressed {comp} ok {bool(torch.equal(decoded, samples))}", flush=True)
c.close()
