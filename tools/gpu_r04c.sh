#!/bin/bash
# Round-4 iteration: parity of the deferred decoder and the encoder, dec_huf_kernel time of the
# product (_ab/libA.so) vs the junk-store diagnostic (libD1), encode A/B certificate on (A) / off (C0),
# decode with deferral off / on.  Every GPU step time-limited.
TAG=${1:-c}
R=${2:-40000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/iter_$TAG.log
: > $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hufjob.py tests/test_gpu_parity.py -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/gpu_subset_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_subset_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_subset_$TAG.log >> $out
for L in A D1; do
  PGN_DEFER_MIN_CHUNKS=1 PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/k2_${TAG}_$L -o run -- python3 tools/codec_timing.py $R 2 > gpurun_out/k2_${TAG}_$L.log 2>&1 || { tail -5 gpurun_out/k2_${TAG}_$L.log; exit 1; }
  f=$(find gpurun_out/k2_${TAG}_$L -name "*kernel_stats.csv" | head -1)
  echo "$L: $(grep -h 'dec_huf_kernel\|dec_zstd_kernel\|dec_merge_kernel\|enc_chunk' $f | cut -d, -f1-4 | tr '\n' ' ')" >> $out
done
for i in 1 2; do
  for L in A C0; do
    echo "enc $L$i: $(PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 120 python3 tools/codec_timing.py $R 4 2>&1 | tail -1)" >> $out || exit 1
  done
done
for d in 1000000 1; do
  echo "defer_min $d: $(PGN_DEFER_MIN_CHUNKS=$d timeout -k 10 120 python3 tools/codec_timing.py 100000 3 2>&1 | tail -1)" >> $out || exit 1
done
cat $out
