#!/bin/bash
# Full GPU suite on the working tree, then A/B timing (_ab/libA.so = HEAD, libB.so = working tree) and
# kernel stats of B.
TAG=${1:-e}
R=${2:-100000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/iter_$TAG.log
: > $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log >> $out
for i in 1 2; do
  for L in A B; do
    echo "$L$i: $(PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 150 python3 tools/codec_timing.py $R 3 2>&1 | tail -1)" >> $out || exit 1
  done
done
PGN_LIB=$PWD/_ab/libB.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 tools/codec_timing.py $R 2 > gpurun_out/prof_$TAG.log 2>&1 || exit 1
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
grep -h 'pgn::' $f | cut -d, -f1-4 >> $out
cat $out
