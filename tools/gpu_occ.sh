#!/bin/bash
# Occupancy slope: encode/decode time vs resident workgroups per CU (PGN_*_WG_PER_CU)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for W in 8 12 16 20; do
  PGN_ENC_WG_PER_CU=$W PGN_DEC_WG_PER_CU=$W timeout -k 10 120 python3 -u tools/codec_timing.py 30000 3 > gpurun_out/occ_$W.log 2>&1 || exit 1
  echo "wg/cu $W: $(tail -1 gpurun_out/occ_$W.log)"
done
