#!/bin/bash
# Deferred sections on the side stream (A) vs on the caller's stream (M); pass size sweep.
TAG=${1:-d}
R=${2:-100000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/iter_$TAG.log
: > $out
PGN_LIB=$PWD/_ab/libA.so timeout -k 10 300 python -u -m pytest tests/test_gpu_hufjob.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/gpu_subset_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_subset_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_subset_$TAG.log >> $out
for i in 1 2; do
  for L in A M; do
    echo "$L$i: $(PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 150 python3 tools/codec_timing.py $R 3 2>&1 | tail -1)" >> $out || exit 1
  done
done
for gG in 16384 50000; do
  echo "A G=$gG: $(PGN_DEFER_G=$gG PGN_LIB=$PWD/_ab/libA.so timeout -k 10 150 python3 tools/codec_timing.py $R 3 2>&1 | tail -1)" >> $out || exit 1
done
cat $out
