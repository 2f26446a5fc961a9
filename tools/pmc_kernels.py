"""Per-kernel SQ / TCP counter summary of the rocprofv3 --pmc passes under a directory (pmc*/).

    python3 tools/pmc_kernels.py DIR [chunks]

Counter values are summed over a kernel's dispatches and printed per chunk (default 20,000 chunks,
tools/gpu_r05_attrib.sh).  The SQ_WAIT_* / SQ_ACTIVE_* / SQ_WAVE_CYCLES counters are quad-cycles
(MI355X_MICROARCH.md): their ratios are the wave-time shares.  Also prints the dispatch's VGPR count
and LDS bytes, and the wave-time shares: waiting (s_waitcnt / barrier), issue-stalled, issuing.
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    return name.split("(")[0].split("::")[-1]


def main():
    d = sys.argv[1]
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[k] = (r.get("VGPR_Count"), r.get("LDS_Block_Size"), r.get("Grid_Size"))
    for k in sorted(agg):
        if not k.startswith(("enc_", "dec_")):
            continue
        v = agg[k]
        print(f"{k}: VGPR {meta[k][0]}, LDS {meta[k][1]} B, grid {meta[k][2]}")
        for c in sorted(v):
            print(f"    {c:32s} {v[c]:16.4g}   per chunk {v[c] / R:12.1f}")
        wc = v.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            sh = {x: v.get(x, 0.0) / wc for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                   "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS")}
            print("    shares of wave time: " + ", ".join(f"{x[3:]} {y:.3f}" for x, y in sh.items() if y))
            if v.get("SQ_BUSY_CYCLES"):
                print(f"    SQ_WAVE_CYCLES / SQ_BUSY_CYCLES = {wc / v['SQ_BUSY_CYCLES']:.1f}")
            if v.get("SQ_WAVES"):
                print(f"    wave-cycles per wave {4 * wc / v['SQ_WAVES']:.0f} (cycles), VALU per wave "
                      f"{v.get('SQ_INSTS_VALU', 0) / v['SQ_WAVES']:.0f}")


if __name__ == "__main__":
    main()
