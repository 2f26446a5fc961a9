#!/bin/bash
# Round-5 evidence of the committed sources: HBM traffic of configs[1] and configs[4] first (so the
# bench lines below carry roofline.traffic for these kernels), GPU tests, smoke, default bench, kernel
# trace of the default bench, configs[4] decode bench.
TAG=${1:-r05}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/traffic.sh $TAG && cp gpurun_out/traffic_$TAG.json profiles/traffic_r05.json \
&& bash tools/traffic.sh ${TAG}_config4 100000 100000 mixed \
&& cp gpurun_out/traffic_${TAG}_config4.json profiles/traffic_r05_config4.json \
&& timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 \
&& timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
&& timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.log 2>&1 \
&& bash tools/profile_run.sh $TAG \
&& timeout -k 10 300 python3 -u bench.py --mixed-pores --decode-only --no-cpu-baseline --no-side \
    > gpurun_out/bench_${TAG}_config4_mixed_decode.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log; tail -1 gpurun_out/bench_$TAG.log | cut -c1-600
tail -1 gpurun_out/bench_${TAG}_config4_mixed_decode.log | cut -c1-400
exit $rc
