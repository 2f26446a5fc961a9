#!/bin/bash
# Round-4 evidence pass: GPU tests, default bench, 2-rank gloo bench, kernel-trace profile of the
# bench, configs[1] traffic, configs[4] decode-only bench + traffic, configs[3] --global-reads line.
TAG=${1:-r04b}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 \
&& timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.log 2>&1 \
&& timeout -k 10 300 python3 -u bench.py --gpus 2 --dist-backend gloo --reads 20000 --no-cpu-baseline \
    > gpurun_out/bench_${TAG}_2rank_gloo.log 2>&1 \
&& bash tools/profile_run.sh $TAG \
&& bash tools/traffic.sh $TAG \
&& cp -r gpurun_out/traffic gpurun_out/traffic_${TAG}_c1 \
&& timeout -k 10 300 python3 -u bench.py --mixed-pores --decode-only --no-cpu-baseline --no-side \
    > gpurun_out/bench_${TAG}_config4_mixed_decode.log 2>&1 \
&& bash tools/traffic.sh ${TAG}_config4 100000 100000 mixed \
&& timeout -k 10 400 python3 -u bench.py --global-reads 1000000 --no-cpu-baseline --no-side \
    > gpurun_out/bench_${TAG}_config3_global.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log; tail -1 gpurun_out/bench_$TAG.log | cut -c1-800
tail -1 gpurun_out/bench_${TAG}_2rank_gloo.log | cut -c1-300
tail -1 gpurun_out/bench_${TAG}_config4_mixed_decode.log | cut -c1-300
tail -1 gpurun_out/bench_${TAG}_config3_global.log | cut -c1-300
exit $rc
