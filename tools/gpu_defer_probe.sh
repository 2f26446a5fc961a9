#!/bin/bash
# Deferred-Huffman decode A/B on one box: codec_timing with the path off / on at several pass sizes,
# then a kernel-trace profile of the deferred decode (per-kernel times).
TAG=${1:-d}
R=${2:-40000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/defer_probe_$TAG.log
: > $out
for cfg in "1000000 32768" "1 32768" "1 16384" "1 8192" "1000000 32768"; do
  set -- $cfg
  echo "PGN_DEFER_MIN_CHUNKS=$1 PGN_DEFER_G=$2" >> $out
  PGN_DEFER_MIN_CHUNKS=$1 PGN_DEFER_G=$2 timeout -k 10 180 python3 -u tools/codec_timing.py $R 3 >> $out 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_defer_$TAG -o run -- \
    python3 tools/codec_timing.py $R 2 > gpurun_out/prof_defer_$TAG.log 2>&1 || exit 1
cat $out
f=$(find gpurun_out/prof_defer_$TAG -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -20
# per-phase wave-cycles of the deferred decode (the _prof library)
PGN_DEFER_MIN_CHUNKS=1 timeout -k 10 200 python -u tools/phase_profile.py 20000 > gpurun_out/phase_defer_$TAG.log 2>&1 || exit 1
tail -40 gpurun_out/phase_defer_$TAG.log
