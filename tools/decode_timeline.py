"""Dispatch timeline of the last decode step in a rocprofv3 kernel trace (start -> end of every decode
kernel, ms from the step's first dispatch): where the step's time goes in the overlapped pipeline.

    python3 tools/decode_timeline.py run_kernel_trace.csv
"""
import csv
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        n = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
    rows.sort()
    last_enc = max((i for i, r in enumerate(rows) if r[2].startswith("enc_")), default=-1)
    dec = [r for r in rows[last_enc + 1:] if r[2].startswith("dec_")]
    if not dec:
        sys.exit("no decode dispatches after the last encode")
    t0 = dec[0][0]
    for a, b, n in dec:
        print(f"{n:18s} {(a - t0) / 1e6:7.3f} -> {(b - t0) / 1e6:7.3f}  ({(b - a) / 1e6:6.3f})")
    zend = max(b for a, b, n in dec if n == "dec_zstd_kernel")
    end = max(b for a, b, n in dec)
    print(f"frame decode ends {(zend - t0) / 1e6:.3f} ms; step ends {(end - t0) / 1e6:.3f} ms "
          f"(drain {(end - zend) / 1e6:.3f} ms)")


if __name__ == "__main__":
    main()
