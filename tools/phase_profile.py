"""Diagnostic: per-phase shader-cycle shares of the encode/decode kernels (PGN_PHASE_PROFILE=1)."""
import ctypes as C
import os
import sys

os.environ.setdefault("PGN_PHASE_PROFILE", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch

from rawnanoporesignalcompression_amd import PGNanoCodec

ENC = ["split", "search", "lit_gather", "hist", "sort", "hdr(writeCTable)", "huf_encode", "raw_lit", "seq",
       "frame_finish", "assemble", "tree_merge", "tree_depth", "tree_maxheight", "tree_canon"]
DEC = ["parse/merge_wait", "huf_table/tab_fill", "fast_path/huf_copy", "unit_fetch", "seq_exec(rest)", "raw_copy", "merge",
       "lit_hdr", "huf_store(passB)", "seq_tables", "seq_bits", "huf_spec(passA)", "huf_sync/tab_stage", "seq_decode",
       "seq_copy", "seq_tail/tab_weights"]
R = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
S = 100000
c = PGNanoCodec(0)
samples, offs, cnt = c.synth_reads(R, S, seed=42)
enc = c.compress_batch(samples, offs, cnt)
if os.environ.get("PGN_ENCODE_ONLY"):  # diagnostic builds whose blobs are not decodable
    torch.cuda.synchronize()
    print("encode ms", c.last_encode_ms())
else:
    out, so, st = c.decompress_batch(enc.blobs, enc.offsets, enc.sizes, cnt)
    torch.cuda.synchronize()
    print("encode ms", c.last_encode_ms(), "decode ms", c.last_decode_ms(), "ok", bool(torch.equal(out, samples)))
buf = np.zeros(128, np.uint64)
c._lib.pgn_debug_phase_cycles(c._h, buf.ctypes.data, 128)
for name, lab, arr in (("encode", ENC, buf[:16]), ("decode", DEC, buf[16:])):
    tot = float(arr.sum())
    print(f"{name}: total {tot/1e9:.2f} Gcycles (summed over waves), per chunk {tot/R/1e3:.1f} kcycles")
    for i, l in enumerate(lab):
        if arr[i]:
            print(f"   {l:18s} {100*arr[i]/tot:6.2f}%  {arr[i]/R/1e3:9.1f} kcyc/chunk")

DCNT = ["huf rounds", "passA overlap iters", "passA bitmap iters", "passA main4 iters", "passA tail iters",
        "sync iters", "sync iters with walks",
        "passB 1-sym iters", "huf tables", "-", "seq blocks", "blocks", "frames", "raw bytes", "-"]
print("decode counters per chunk:")
for i, l in enumerate(DCNT):
    if buf[48 + i]:
        print(f"   {l:24s} {buf[48 + i] / R:12.2f}")
ECNT = ["search rounds", "sequences found", "tree builds", "tree merge rounds", "depth iters", "writeCTable",
        "ctable symbols", "huf encode steps", "hist iters", "split steps", "seq sections", "seqs encoded",
        "frames", "blocks", "search same-slot iters", "-"]
print("encode counters per chunk:")
for i, l in enumerate(ECNT):
    if buf[32 + i]:
        print(f"   {l:24s} {buf[32 + i] / R:12.2f}")

HUF = ["tables (job flags, compact tables to LDS)", "setup + 8-iteration prologue", "trips of 8 iterations",
       "drain, head/tail bytes, last symbols, end check"]
hp, hc = buf[64:80], buf[96:112]
tot = float(hp.sum())
if tot:
    print(f"dec_huf_kernel: total {tot/1e9:.2f} Gcycles (summed over waves), per chunk {tot/R/1e3:.1f} kcycles")
    for i, l in enumerate(HUF):
        print(f"   {l:48s} {100*hp[i]/tot:6.2f}%  {hp[i]/R/1e3:9.1f} kcyc/chunk")
    waves = max(int(hc[0]), 1)
    print(f"   waves {waves}, trips per wave {hc[1]/waves:.1f}, live lanes per wave {hc[2]/waves:.1f}, "
          f"symbols per chunk {hc[3]/R:.0f}, wave-cycles per wave {tot/waves/1e3:.1f} k, "
          f"per trip {hp[2]/max(hc[1],1):.0f}")
