#!/bin/bash
# dec_huf_kernel diagnostics: kernel time of the product build (A) and of the PGN_K2_DIAG builds
# (D1 junk stores, D2 one-block loads, D3 no table read; tools/ab_k2diag.sh), then one PMC pass of A.
TAG=${1:-k2}
R=${2:-40000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PGN_DEFER_MIN_CHUNKS=1
for L in ${LIBS:-A D1 D2 D3}; do
  PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k2_${TAG}_$L -o run -- \
      python3 tools/codec_timing.py $R 2 > gpurun_out/k2_${TAG}_$L.log 2>&1 || { tail -5 gpurun_out/k2_${TAG}_$L.log; exit 1; }
  f=$(find gpurun_out/k2_${TAG}_$L -name "*kernel_stats.csv" | head -1)
  echo "$L: $(grep -h 'dec_huf_kernel\|dec_zstd_kernel' $f | cut -d, -f1-4 | tr '\n' ' ')"
done
PGN_LIB=$PWD/_ab/libA.so timeout -s KILL 120 rocprofv3 --kernel-trace \
    --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU \
    --output-format csv -d gpurun_out/k2_${TAG}_pmc -o run -- python3 tools/codec_timing.py 20000 1 > gpurun_out/k2_${TAG}_pmc.log 2>&1 || { tail -5 gpurun_out/k2_${TAG}_pmc.log; exit 1; }
f=$(find gpurun_out/k2_${TAG}_pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r.get("Kernel_Name", "")
    if "dec_huf" not in k and "dec_zstd" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k[:40], {c: f"{v:.4g}" for c, v in sorted(d.items())})
PY
