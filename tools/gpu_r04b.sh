#!/bin/bash
# Round-4 iteration pass: parity subset (encoder blobs vs the oracle, deferred decoder), codec timing
# with the deferred decode off / on, kernel-trace stats, phase cycles -- every step time-limited.
TAG=${1:-b}
R=${2:-40000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/iter_$TAG.log
: > $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hufjob.py tests/test_gpu_multiblock.py -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/gpu_subset_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_subset_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_subset_$TAG.log >> $out
for cfg in "1000000 32768" "1 32768" "1 16384"; do
  set -- $cfg
  echo "PGN_DEFER_MIN_CHUNKS=$1 PGN_DEFER_G=$2" >> $out
  PGN_DEFER_MIN_CHUNKS=$1 PGN_DEFER_G=$2 timeout -k 10 180 python3 -u tools/codec_timing.py $R 3 >> $out 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_iter_$TAG -o run -- \
    python3 tools/codec_timing.py $R 2 > gpurun_out/prof_iter_$TAG.log 2>&1 || exit 1
PGN_DEFER_MIN_CHUNKS=1 timeout -k 10 200 python -u tools/phase_profile.py 20000 > gpurun_out/phase_iter_$TAG.log 2>&1 || exit 1
cat $out
f=$(find gpurun_out/prof_iter_$TAG -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | grep "pgn::" | head -12
tail -42 gpurun_out/phase_iter_$TAG.log
