#!/bin/bash
# One GPU-box pass (run via gpurun): parity tests, default bench, the --gpus 2 launcher rehearsed with
# two gloo ranks on the box's one GPU, kernel-trace profile, HBM traffic + L2 hit rate.
# Every GPU step has its own time limit; the steps are chained so the first failure ends the call.
TAG=${1:-latest}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 \
&& timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.log 2>&1 \
&& timeout -k 10 300 python3 -u bench.py --gpus 2 --dist-backend gloo --reads 20000 --no-cpu-baseline \
    > gpurun_out/bench_${TAG}_2rank_gloo.log 2>&1 \
&& bash tools/profile_run.sh $TAG \
&& bash tools/traffic.sh $TAG
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log; tail -1 gpurun_out/bench_$TAG.log | cut -c1-600
tail -1 gpurun_out/bench_${TAG}_2rank_gloo.log | cut -c1-300
exit $rc
