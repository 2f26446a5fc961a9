#!/bin/bash
# PMC probe of the codec kernels on a small batch (run on the GPU box).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export PGN_PHASE_PROFILE=0
R=${1:-5000}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/trace -o run -- \
    python3 tools/phase_profile.py $R > gpurun_out/pmc/trace.log 2>&1
SETS=${PMC_SETS:-all}
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQC_DCACHE_HITS SQC_DCACHE_MISSES"; do
  N=$(echo $SET | cut -d' ' -f1)
  [ "$SETS" = all ] || [[ " $SETS " == *" $N "* ]] || continue
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d gpurun_out/pmc/$N -o run -- \
      python3 tools/phase_profile.py $R > gpurun_out/pmc/$N.log 2>&1 || echo "pass $N failed"
done
