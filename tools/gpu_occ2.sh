#!/bin/bash
# Decode occupancy slope with and without the side-stream merge (PGN_DIAG_NO_MERGE: timing only)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for NM in 0 1; do
  for W in 8 12 16 20; do
    PGN_DIAG_NO_MERGE=$NM PGN_DEC_WG_PER_CU=$W timeout -k 10 120 python3 -u tools/codec_timing.py 30000 3 > gpurun_out/occ2_${NM}_$W.log 2>&1 || exit 1
    echo "no_merge $NM wg/cu $W: $(tail -1 gpurun_out/occ2_${NM}_$W.log)"
  done
done
