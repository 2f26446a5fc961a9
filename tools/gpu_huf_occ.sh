#!/bin/bash
# dec_huf / dec_merge probes (run via gpurun): serial diagnostic builds (_ab/lib*.so, tools/ab_defs.sh
# NAME -DPGN_SERIAL_DECODE ...) against the serial product build (_ab/libSER.so): PGN_K2_DIAG=4 with
# PGN_K2_PAD (256-entry tables, LDS padded: occupancy), PGN_K2_DIAG=1/2/3 (junk stores / one-block
# loads / no table read), PGN_MERGE_DIAG=1 (L2-resident intermediate reads).  Kernel trace of one
# 20,000-chunk decode call each; prints each decode kernel's duration and dec_huf's LDS allocation.
TAG=${1:-r05_hufocc}
# LIBS may repeat a name (interleaved repeats); outputs k_<lib>_<i>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
rm -rf $O && mkdir -p $O
i=0
for L in ${LIBS:-SER D8 D12}; do
  i=$((i + 1)); K=k_${L}_$i
  PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/$K -o run -- \
      python3 tools/codec_timing.py 20000 1 > $O/$K.log 2>&1 || { tail -3 $O/$K.log; exit 1; }
  echo "$L: $(python3 tools/decode_wall.py $O/$K/run_kernel_trace.csv | tail -1 | cut -d: -f2-)"
  python3 - $O/$K/run_kernel_trace.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dec_huf" in r["Kernel_Name"]:
        print("   dec_huf LDS", r.get("LDS_Block_Size", r.get("Lds_Size", "?")), "VGPR", r.get("VGPR_Count", r.get("Arch_VGPR_Count", "?")))
        break
PY
done
