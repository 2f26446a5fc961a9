#!/bin/bash
# Interleaved A/B at the bench's size (100,000 chunks: several decode passes): bash tools/gpu_ab_bench.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-abb}
mkdir -p gpurun_out
for i in 1 2; do
  for L in ${LIBS:-A B}; do
    PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 200 python3 -u tools/codec_timing.py 100000 3 > gpurun_out/abb_${TAG}_$L$i.log 2>&1 || { tail -3 gpurun_out/abb_${TAG}_$L$i.log; exit 1; }
    echo "$L$i: $(tail -1 gpurun_out/abb_${TAG}_$L$i.log)"
  done
done
