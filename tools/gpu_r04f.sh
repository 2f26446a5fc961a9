#!/bin/bash
# A/B: B (LUT merge), N (bit-select merge), P (LUT merge, K2 prefetch 2); isolated kernel times
# (serial builds S1 = LUT merge, S0 = bit-select merge).
TAG=${1:-f}
R=${2:-100000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/iter_$TAG.log
: > $out
PGN_LIB=$PWD/_ab/libP.so timeout -k 10 300 python -u -m pytest tests/test_gpu_hufjob.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/gpu_subset_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_subset_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_subset_$TAG.log >> $out
for i in 1 2; do
  for L in ${LIBS:-B N P}; do
    echo "$L$i: $(PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 150 python3 tools/codec_timing.py $R 3 2>&1 | tail -1)" >> $out || exit 1
  done
done
for L in S1 S0; do
  PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$L -o run -- \
      python3 tools/codec_timing.py 40000 2 > gpurun_out/prof_${TAG}_$L.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_${TAG}_$L -name "*kernel_stats.csv" | head -1)
  echo "$L: $(tail -1 gpurun_out/prof_${TAG}_$L.log)" >> $out
  grep -h 'pgn::dec\|pgn::enc' $f | cut -d, -f1-4 >> $out
done
cat $out
