#!/bin/bash
# GPU tests (both Huffman decoders), codec timing A/B and phase profiles (run via gpurun).
TAG=${1:-m}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; exit $rc; }
PGN_HUF=seg timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_${TAG}_seg.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_${TAG}_seg.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_${TAG}_seg.log | head -20; exit $rc; }
for H in twopass seg; do
  PGN_HUF=$H timeout -k 10 120 python3 tools/codec_timing.py 30000 3 > gpurun_out/timing_${TAG}_$H.log 2>&1 || exit 1
  echo "$H: $(tail -1 gpurun_out/timing_${TAG}_$H.log)"
done
timeout -k 10 200 python -u tools/phase_profile.py 20000 > gpurun_out/phase_${TAG}.log 2>&1 || exit 1
sed -n '/^decode:/,/^decode counters/p' gpurun_out/phase_${TAG}.log
