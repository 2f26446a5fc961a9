"""Per-step encode / decode walls and per-kernel busy time from a rocprofv3 kernel trace.

    python3 tools/decode_wall.py run_kernel_trace.csv [chunks_per_step]

A step's decode is the run of dispatches named dec_* between two encode dispatches (enc_*); its wall
is the last end minus the first start.  For each kernel the sum of its dispatch durations in the
step is printed beside it: with overlapped streams those sums exceed the wall, in a serial build
(PGN_SERIAL_DECODE) they add up to it.
"""
import collections
import csv
import sys


def short(name):
    return name.split("(")[0].split("::")[-1].split("<")[0]


def main():
    path = sys.argv[1]
    per_step_chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    groups = []  # (direction, [rows])
    for r in rows:
        k = r[2]
        d = "dec" if k.startswith(("dec_", "vbz_parse", "vbz_merge")) else ("enc" if k.startswith(("enc_", "vbz_split", "vbz_assemble")) else None)
        if d is None:
            continue
        if not groups or groups[-1][0] != d:
            groups.append((d, []))
        groups[-1][1].append(r)
    for i, (d, g) in enumerate(groups):
        wall = (max(x[1] for x in g) - min(x[0] for x in g)) / 1e6
        busy = collections.OrderedDict()
        cnt = collections.Counter()
        for s, e, k in g:
            busy[k] = busy.get(k, 0.0) + (e - s) / 1e6
            cnt[k] += 1
        parts = ", ".join(f"{k} {v:.3f} ms x{cnt[k]}" for k, v in busy.items())
        extra = f"  ({per_step_chunks / wall / 1e3:.1f} Mchunks/s)" if per_step_chunks else ""
        print(f"step-part {i:2d} {d}: wall {wall:8.3f} ms, kernel sum {sum(busy.values()):8.3f} ms{extra}: {parts}")


if __name__ == "__main__":
    main()
