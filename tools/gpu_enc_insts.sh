#!/bin/bash
# Encode instruction counts per chunk by phase (run via gpurun): one PMC pass (SQ_INSTS_VALU / SALU /
# LDS) over a 20,000-chunk encode for each library LIBS="E0 E1 ..." (_ab/lib*.so; the PGN_AB_SKIP
# diagnostic builds stop the zstd stage after successive phases, so differences are per phase).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-encinsts}
mkdir -p $O
R=20000
for n in $LIBS; do
  PGN_ENCODE_ONLY=1 PGN_LIB=$PWD/_ab/lib$n.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
      --output-format csv -d $O/$n -o run -- python3 tools/phase_profile.py $R > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  python3 - "$O/$n" "$n" "$R" <<'PY'
import csv, glob, sys, collections
d, n, R = sys.argv[1], sys.argv[2], int(sys.argv[3])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(agg):
    v = agg[k]
    if k.startswith("enc_") and v["SQ_INSTS_VALU"] > 1e6:
        print(f"{n} {k}: VALU {v['SQ_INSTS_VALU']/R/1e3:.1f}k SALU {v['SQ_INSTS_SALU']/R/1e3:.1f}k LDS {v['SQ_INSTS_LDS']/R/1e3:.1f}k "
              f"LDS bank-conflict cycles {v['SQ_LDS_BANK_CONFLICT']/R/1e3:.1f}k active LDS cycles {v['SQ_ACTIVE_INST_LDS']/R/1e3:.1f}k per chunk")
PY
done
