#!/bin/bash
# Phase cycles (profile build) and instruction counts (PMC) of the current kernels, 20,000 chunks.
TAG=${1:-h}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/phase_profile.py 20000 > gpurun_out/phase_$TAG.log 2>&1 || exit 1
for SET in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"; do
  N=$(echo $SET | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d gpurun_out/pmc_${TAG}_$N -o run -- \
      python3 tools/codec_timing.py 20000 1 > gpurun_out/pmc_${TAG}_$N.log 2>&1 || exit 1
done
python3 - gpurun_out/pmc_${TAG}_SQ_INSTS_VALU gpurun_out/pmc_${TAG}_SQ_WAVES <<'PY'
import csv, sys, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if "pgn::" not in k: continue
            agg[k.split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: f"{v / 40000:.4g}" for c, v in sorted(d.items())}, "(per chunk)")
PY
head -40 gpurun_out/phase_$TAG.log
