"""Summarise tools/pmc_probe.sh output: per-kernel duration and counters (per launch-set totals)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
stats = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))
if stats:
    print("kernel durations:")
    for r in csv.DictReader(open(stats[0])):
        print(f"  {r['Name'][:40]:40s} calls {r['Calls']:>6s} total {float(r['TotalDurationNs'])/1e6:9.3f} ms avg {float(r['AverageNs'])/1e3:9.1f} us")
agg = collections.defaultdict(dict)
for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-28:]
        agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
names = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU",
         "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM",
         "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_INST_CYCLES_VMEM_RD",
         "SQC_ICACHE_HITS", "SQC_ICACHE_MISSES", "SQC_ICACHE_MISSES_DUPLICATE", "SQ_IFETCH", "SQC_DCACHE_HITS",
         "SQC_DCACHE_MISSES"]
for k, v in sorted(agg.items()):
    if "pgn" not in k and "enc_" not in k and "dec_" not in k:
        continue
    print(k)
    for n in names:
        if n in v:
            print(f"   {n:26s} {v[n]:16.0f}")
