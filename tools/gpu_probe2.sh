#!/bin/bash
# timing A/B + merge phase profile + PMC comparison of the two Huffman decoders (run via gpurun)
TAG=${1:-p2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for H in twopass seg; do
  PGN_HUF=$H timeout -k 10 120 python3 tools/codec_timing.py 30000 3 > gpurun_out/timing_${TAG}_$H.log 2>&1 || exit 1
  echo "$H: $(tail -1 gpurun_out/timing_${TAG}_$H.log)"
done
timeout -k 10 200 python -u tools/phase_profile.py 20000 > gpurun_out/phase_${TAG}.log 2>&1 || exit 1
grep -E "merge|huf_" gpurun_out/phase_${TAG}.log | head -8
bash tools/pmc_seg.sh 10000 2>&1 | tail -3
