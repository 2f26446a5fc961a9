#!/bin/bash
# Instruction counts per chunk of the codec kernels for each library build under ab/*.so (run via
# gpurun): one rocprofv3 PMC pass (SQ_INSTS_VALU / SALU / LDS) over a 20,000-chunk encode+decode.
# The environment passes through (PGN_ENC_PIPELINE=staged splits the encode into its three kernels).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abi
R=${1:-20000}
for v in ab/*.so; do
  n=$(basename $v .so)
  PGN_LIB=$PWD/$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES \
      --output-format csv -d gpurun_out/abi/$n -o run -- python3 tools/phase_profile.py $R > gpurun_out/abi/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abi/$n.log; exit 1; }
  python3 - "$n" "$R" <<'PY'
import csv, glob, sys, collections
n, R = sys.argv[1], int(sys.argv[2])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"gpurun_out/abi/{n}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
out = []
for k in sorted(agg):
    v = agg[k]
    if v['SQ_INSTS_VALU'] > 1e6:
        out.append(f"{k}: V {v['SQ_INSTS_VALU']/R/1e3:.1f}k S {v['SQ_INSTS_SALU']/R/1e3:.1f}k L {v['SQ_INSTS_LDS']/R/1e3:.1f}k")
print(n, " | ".join(out))
PY
done
