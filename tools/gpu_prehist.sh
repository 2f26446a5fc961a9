#!/bin/bash
# Encode histograms counted in the split (round 5): parity of the working-tree library (C) and of its
# exact-sizes build (X), phase profiles of HEAD (A) and C, interleaved bench-size A/B/C.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for L in ${TLIBS:-C}; do
  PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/ph_tests$L.log 2>&1 || { tail -20 gpurun_out/ph_tests$L.log; exit 1; }
  tail -1 gpurun_out/ph_tests$L.log
done
for L in ${PLIBS:-A C}; do
  PGN_PHASE_PROFILE=1 PGN_LIB=$PWD/_ab/lib${L}_prof.so timeout -k 10 200 python -u tools/phase_profile.py 20000 \
      > gpurun_out/ph_phase_$L.log 2>&1 || { tail -5 gpurun_out/ph_phase_$L.log; exit 1; }
  grep -A16 "^encode:" gpurun_out/ph_phase_$L.log
done
LIBS="${ABLIBS:-A B C}" bash tools/gpu_ab_bench.sh prehist2
