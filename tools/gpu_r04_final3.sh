#!/bin/bash
# Pass-size confirmation (env overrides) and the evidence of the sources with the new default:
# GPU tests, default bench, configs[1] / configs[4] traffic, configs[4] bench.
TAG=${1:-r04c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
GS="25000 16667 25000 16667" bash tools/gpu_defer_sweep.sh $TAG | tee gpurun_out/defer_sweep_$TAG.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 \
&& timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.log 2>&1 \
&& bash tools/profile_run.sh $TAG \
&& bash tools/traffic.sh $TAG \
&& timeout -k 10 300 python3 -u bench.py --mixed-pores --decode-only --no-cpu-baseline --no-side \
    > gpurun_out/bench_${TAG}_config4_mixed_decode.log 2>&1 \
&& bash tools/traffic.sh ${TAG}_config4 100000 100000 mixed
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log; tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
tail -1 gpurun_out/bench_${TAG}_config4_mixed_decode.log | cut -c1-300
exit $rc
