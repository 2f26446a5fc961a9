"""Timeline of steady-state per-chunk calls from a rocprofv3 trace directory (kernel, memory-copy and
HIP-API traces): where a pgn_compress_signal / pgn_decompress_signal call's time goes."""
import csv
import glob
import os
import sys

d = sys.argv[1]
ev = []
for kind, pat, name in (("K", "*kernel_trace.csv", "Kernel_Name"), ("C", "*memory_copy_trace.csv", "Direction"),
                        ("A", "*hip_api_trace.csv", "Function")):
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r.get(name) or r.get("Operation") or "?"
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, n.split("(")[0][-40:]))
ev.sort()
# find API calls of hipStreamSynchronize: each per-chunk call ends with one; print the 3 calls around the middle
syncs = [e for e in ev if e[2] == "A" and "StreamSynchronize" in e[3]]
mid = len(syncs) // 2
for s_end_idx in (mid, mid + 1, len(syncs) - 3):
    t1 = syncs[s_end_idx][1]
    t0 = syncs[s_end_idx - 1][1]
    print(f"--- call ending at sync #{s_end_idx}: {(t1 - t0) / 1e3:.1f} us")
    for e in ev:
        if t0 <= e[0] <= t1:
            print(f"  {(e[0] - t0) / 1e3:8.1f} .. {(e[1] - t0) / 1e3:8.1f} us  {e[2]} {e[3]}")
