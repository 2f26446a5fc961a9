#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "16 12 2" "16 12 4" "16 12 8" "12 10 4" "20 16 4"; do
  set -- $cfg
  PARTS=$3 PGN_ENC_WG_PER_CU=$1 PGN_DEC_WG_PER_CU=$2 timeout -k 10 150 python3 tools/overlap_timing.py 100000 > gpurun_out/overlap_$1_$2_$3.log 2>&1 || exit 1
  echo "enc $1 dec $2 parts $3: $(grep step gpurun_out/overlap_$1_$2_$3.log | tr '\n' ' ')"
done
