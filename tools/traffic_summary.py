"""Per-kernel HBM bytes of one bench step from tools/traffic.sh's two PMC passes.

FETCH_SIZE and WRITE_SIZE are rocprofv3 derived counters in KiB, built from the L2 memory-side
request counters (TCC_EA0_RDREQ / _WRREQ).  MI355X_MICROARCH.md ("HBM [CDNA4]"): on gfx950
FETCH_SIZE reports exactly half the bytes of wide coalesced streaming reads, so it is doubled here;
WRITE_SIZE is taken as is.  Both raw and corrected values are written."""
import collections
import csv
import glob
import json
import os
import sys

d, R, S, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
workload = sys.argv[5] if len(sys.argv) > 5 else "configs[1]"
val = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split()[-1].split("::")[-1]
        val[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k][r["Counter_Name"]] += 1
stages = {"c5_encode": ["enc_split_kernel", "enc_zstd_kernel", "enc_assemble_kernel"],
          "c5_decode": ["dec_parse_kernel", "dec_zstd_kernel", "dec_merge_kernel"]}
if "dec_huf_kernel" in val:  # large batches: the deferred Huffman sections
    stages["c5_decode"].insert(2, "dec_huf_kernel")
# the fused per-chunk kernels (the default encode path) stand for their whole direction
if "enc_chunk_kernel<0>" in val:
    stages["c5_encode"] = ["enc_chunk_kernel<0>"]
if "dec_chunk_kernel<0>" in val:
    stages["c5_decode"] = ["dec_chunk_kernel<0>"]
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import source_digest  # noqa: E402  (the kernel sources this measurement belongs to)

res = {"reads": R, "samples": S, "workload": workload, "unit": "bytes per stage launch (one direction over the whole batch)",
       "source_sha256": source_digest(),
       "correction": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section)", "kernels": {}}
for k, v in val.items():
    if not any(k.startswith(p) for p in ("enc_", "dec_")):
        continue
    fetch, write = v.get("FETCH_SIZE", 0.0) * 1024, v.get("WRITE_SIZE", 0.0) * 1024
    hit, miss = v.get("TCC_HIT_sum", 0.0), v.get("TCC_MISS_sum", 0.0)
    res["kernels"][k] = {"fetch_raw": fetch, "write": write, "bytes": 2 * fetch + write,
                         "dispatches": calls[k].get("FETCH_SIZE", 0),
                         "tcc_hit": hit, "tcc_miss": miss,
                         "l2_hit_rate": round(hit / (hit + miss), 4) if hit + miss > 0 else None}
for st, ks in stages.items():
    if all(k in res["kernels"] for k in ks):
        res[st] = sum(res["kernels"][k]["bytes"] for k in ks)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
