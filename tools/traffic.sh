#!/bin/bash
# HBM traffic and L2 hit rate of one bench step, per kernel (run on the GPU box).  Separate --pmc passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950: MI355X_MICROARCH.md "rocprofv3 PMC
# slots"), then tools/traffic_summary.py applies the guide's gfx950 FETCH_SIZE correction and
# writes gpurun_out/traffic_<tag>.json; copied to profiles/, bench.py reads it into roofline.traffic.
set -e
TAG=${1:-latest}
R=${2:-100000}
S=${3:-100000}
MODE=${4:-default}   # "mixed": configs[4]'s corpus (tools/traffic_probe.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/traffic
mkdir -p gpurun_out/traffic
# third pass: L2 hit/miss (TCC_HIT_sum / TCC_MISS_sum, 2 of the 4 TCC slots)
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  D=${C%% *}
  timeout -s KILL 400 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/traffic/$D -o run -- \
      python3 tools/traffic_probe.py $R $S $MODE > gpurun_out/traffic/$D.log 2>&1
done
python3 tools/traffic_summary.py gpurun_out/traffic $R $S gpurun_out/traffic_$TAG.json \
    $([ "$MODE" = mixed ] && echo "configs[4]" || echo "configs[1]")  # copied into profiles/ to commit
