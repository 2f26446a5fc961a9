#!/bin/bash
# A/B timing of _ab/libA.so vs _ab/libB.so, interleaved: bash tools/gpu_ab2.sh TAG [READS]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-ab}; R=${2:-30000}
mkdir -p gpurun_out
for i in 1 2; do
  for L in ${LIBS:-A B}; do
    PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 120 python3 -u tools/codec_timing.py $R 5 > gpurun_out/ab_${tag}_$L$i.log 2>&1 || { tail -3 gpurun_out/ab_${tag}_$L$i.log; exit 1; }
    echo "$L$i: $(tail -1 gpurun_out/ab_${tag}_$L$i.log)"
  done
done
