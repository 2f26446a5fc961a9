#!/bin/bash
# Quick segmented-decoder probe (run via gpurun): codec timing A/B and the seg phase profile.
TAG=${1:-segq}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for H in twopass seg; do
  PGN_HUF=$H timeout -k 10 120 python3 tools/codec_timing.py 30000 3 > gpurun_out/timing_${TAG}_$H.log 2>&1 || exit 1
  echo "$H: $(tail -1 gpurun_out/timing_${TAG}_$H.log)"
done
PGN_HUF=seg timeout -k 10 200 python -u tools/phase_profile.py 20000 > gpurun_out/phase_${TAG}_seg.log 2>&1 || exit 1
sed -n '/^decode:/,/^encode counters/p' gpurun_out/phase_${TAG}_seg.log
