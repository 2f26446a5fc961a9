#!/bin/bash
# PMC comparison of the decode zstd kernel, two-pass vs segmented Huffman decoder (run via gpurun).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pmcseg
mkdir -p $OUT
R=${1:-10000}
for H in twopass seg; do
  for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" \
             "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAVES" \
             "TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TD_BUSY_avr"; do
    N=$(echo $SET | cut -d' ' -f1)
    PGN_HUF=$H timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $OUT/${H}_$N -o run -- \
        python3 tools/codec_timing.py $R 1 > $OUT/${H}_$N.log 2>&1 || { echo "pass $H $N failed"; tail -3 $OUT/${H}_$N.log; }
  done
done
python3 - $OUT $R <<'PY'
import csv, glob, sys, collections
out, R = sys.argv[1], int(sys.argv[2])
for H in ("twopass", "seg"):
    agg = collections.defaultdict(float)
    for f in glob.glob(f"{out}/{H}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "dec_zstd_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(H, " ".join(f"{k}={v/R:.0f}" for k, v in sorted(agg.items())))
PY
