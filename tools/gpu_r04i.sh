#!/bin/bash
# Zero-copy raw frames: new + decode parity tests on the working tree, then A/B timing vs HEAD.
TAG=${1:-i}
R=${2:-100000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/iter_$TAG.log
: > $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_zero_copy.py tests/test_gpu_hufjob.py tests/test_gpu_parity.py \
    tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_subset_$TAG.log 2>&1 \
    || { tail -40 gpurun_out/gpu_subset_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_subset_$TAG.log >> $out
for i in 1 2; do
  for L in A B; do
    echo "$L$i: $(PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 150 python3 tools/codec_timing.py $R 3 2>&1 | tail -1)" >> $out || exit 1
  done
done
cat $out
