"""Per-kernel total duration (ms) from a rocprofv3 kernel-trace CSV directory (tools/*.sh output)."""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        continue
    tot = collections.Counter()
    cnt = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
        tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        cnt[k] += 1
    print(d)
    for k, v in tot.most_common(10):
        print(f"   {k:40s} {cnt[k]:5d} calls {v:9.3f} ms")
