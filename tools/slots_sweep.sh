#!/bin/bash
# Encode/decode time vs resident zstd workgroups per CU (run via gpurun).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for E in 16 14 12 10 8; do
  PGN_ENC_WG_PER_CU=$E PGN_DEC_WG_PER_CU=$E timeout -k 10 120 python3 tools/codec_timing.py 30000 3 > gpurun_out/sweep_$E.log 2>&1 || exit 1
  echo "wg/cu $E: $(tail -1 gpurun_out/sweep_$E.log)"
done
