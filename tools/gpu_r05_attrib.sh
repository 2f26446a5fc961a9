#!/bin/bash
# Decode attribution (run via gpurun): isolated per-kernel times of the bench-size decode from a serial
# build (every decode kernel on the caller's stream, _ab/libSER.so = tools/ab_defs.sh SER
# -DPGN_SERIAL_DECODE), the production trace's decode wall, SQ counter passes over one 20,000-chunk
# decode pass per kernel, and the phase profile of the serial build (_ab/libSERP.so, with PGN_PROFILE).
# Outputs under gpurun_out/$TAG/.
TAG=${1:-r05a}
R=${2:-100000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
rm -rf $O && mkdir -p $O
run_trace() {  # name lib
  PGN_LIB=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1 -o run -- \
      python3 tools/codec_timing.py $R 1 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; return 1; }
  python3 tools/decode_wall.py $O/$1/run_kernel_trace.csv $R > $O/$1_walls.txt && tail -4 $O/$1_walls.txt
}
run_trace ser $PWD/_ab/libSER.so && run_trace prod $PWD/rawnanoporesignalcompression_amd/_build/libpgnano_hip.so || exit 1
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
have() { grep -qw "$1" $O/counters.txt; }
P=1
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
  cs=""
  for c in $set; do have ${c%_sum} && cs="$cs $c"; done
  [ -z "$cs" ] && continue
  echo "pass $P:$cs"
  PGN_LIB=$PWD/_ab/libSER.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $cs --output-format csv -d $O/pmc$P -o run -- \
      python3 tools/codec_timing.py 20000 0 > $O/pmc$P.log 2>&1 || { echo "pmc pass $P failed"; tail -5 $O/pmc$P.log; exit 1; }
  P=$((P + 1))
done
python3 tools/pmc_kernels.py $O > $O/pmc_kernels.txt && cat $O/pmc_kernels.txt
PGN_LIB=$PWD/_ab/libSERP.so timeout -k 10 200 python3 -u tools/phase_profile.py 20000 > $O/phase.log 2>&1 || { tail -5 $O/phase.log; exit 1; }
tail -30 $O/phase.log
