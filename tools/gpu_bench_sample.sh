#!/bin/bash
# One more sample of the default bench line and the configs[4] decode line on whichever box gpurun
# gives (box-to-box spread of the same sources): bash tools/gpu_bench_sample.sh TAG
TAG=${1:-sample}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.log 2>&1 \
&& timeout -k 10 300 python3 -u bench.py --mixed-pores --decode-only --no-cpu-baseline --no-side \
    > gpurun_out/bench_${TAG}_config4_mixed_decode.log 2>&1
rc=$?
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300; tail -1 gpurun_out/bench_${TAG}_config4_mixed_decode.log | cut -c1-200
exit $rc
