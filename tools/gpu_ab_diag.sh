#!/bin/bash
# Phase profiles and dec_zstd/dec_merge PMC counters of _ab/libA vs _ab/libB (run via gpurun):
# bash tools/gpu_ab_diag.sh TAG [READS]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-diag}; R=${2:-20000}
mkdir -p gpurun_out/abd
for L in A B; do
  PGN_PHASE_PROFILE=1 PGN_LIB=$PWD/_ab/lib${L}_prof.so timeout -k 10 120 python3 -u tools/phase_profile.py $R \
      > gpurun_out/abd/phase_${tag}_$L.log 2>&1 || { tail -3 gpurun_out/abd/phase_${tag}_$L.log; exit 1; }
done
for L in A B; do
  PGN_LIB=$PWD/_ab/lib$L.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
      --output-format csv -d gpurun_out/abd/pmc_${tag}_$L -o run -- python3 tools/phase_profile.py $R \
      > gpurun_out/abd/pmc_${tag}_$L.log 2>&1 || { echo "pmc $L failed"; tail -3 gpurun_out/abd/pmc_${tag}_$L.log; exit 1; }
done
python3 - "$tag" "$R" <<'PY'
import csv, glob, sys, collections
tag, R = sys.argv[1], int(sys.argv[2])
for L in "AB":
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"gpurun_out/abd/pmc_{tag}_{L}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k in sorted(agg):
        if k.startswith(("enc_", "dec_")):
            print(L, k, " ".join(f"{c}={x/R/1e3:.1f}k" for c, x in sorted(agg[k].items())))
PY
for L in A B; do echo "== $L"; grep -A12 "^decode:" gpurun_out/abd/phase_${tag}_$L.log; done
