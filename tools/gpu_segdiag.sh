#!/bin/bash
# timing of the one-pass decoder with diagnostic switches (wrong output; timing only)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for D in 0 4 5 6 7; do
  PGN_HUF=seg PGN_SEG_DIAG=$D timeout -k 10 120 python3 tools/codec_timing.py 30000 3 > gpurun_out/timing_diag$D.log 2>&1 || exit 1
  echo "diag $D: $(tail -1 gpurun_out/timing_diag$D.log)"
done
PGN_HUF=twopass timeout -k 10 120 python3 tools/codec_timing.py 30000 3 > gpurun_out/timing_diagtp.log 2>&1 || exit 1
echo "twopass: $(tail -1 gpurun_out/timing_diagtp.log)"
