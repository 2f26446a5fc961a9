#!/bin/bash
# Evidence of the committed sources (run via gpurun): HBM traffic of configs[1] and configs[4] first
# (copied to profiles/traffic_$ROUND.json and traffic_${ROUND}_config4.json, which bench.py reads into
# roofline.traffic when their source digest matches), GPU tests, smoke, default bench, kernel trace of
# the default bench and its decode timeline, configs[4] decode bench; with EXTRA=1 also the configs[2]
# (R10.4.1, VBZ ratio) and configs[3] (1,000,000 distinct reads) lines and the --gpus 2 launcher
# rehearsed with two gloo ranks on the box's one GPU.   ROUND=r06 bash tools/gpu_final.sh TAG
TAG=${1:-final}
ROUND=${ROUND:-r06}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/traffic.sh $TAG && cp gpurun_out/traffic_$TAG.json profiles/traffic_$ROUND.json \
&& bash tools/traffic.sh ${TAG}_config4 100000 100000 mixed \
&& cp gpurun_out/traffic_${TAG}_config4.json profiles/traffic_${ROUND}_config4.json \
&& timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 \
&& timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
&& timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.log 2>&1 \
&& bash tools/profile_run.sh $TAG \
&& python3 tools/decode_timeline.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/timeline_$TAG.txt \
&& timeout -k 10 300 python3 -u bench.py --mixed-pores --decode-only --no-cpu-baseline --no-side \
    > gpurun_out/bench_${TAG}_config4_mixed_decode.log 2>&1
rc=$?
if [ $rc = 0 ] && [ "${EXTRA:-0}" = 1 ]; then
  timeout -k 10 300 python3 -u bench.py --pore r1041 --compare-vbz --no-cpu-baseline --no-side \
      > gpurun_out/bench_${TAG}_config2_r1041_vs_vbz.log 2>&1 \
  && timeout -k 10 400 python3 -u bench.py --global-reads 1000000 --no-cpu-baseline --no-side \
      > gpurun_out/bench_${TAG}_config3_global.log 2>&1 \
  && timeout -k 10 300 python3 -u bench.py --gpus 2 --dist-backend gloo --reads 20000 --no-cpu-baseline \
      > gpurun_out/bench_${TAG}_2rank_gloo.log 2>&1
  rc=$?
  for f in config2_r1041_vs_vbz config3_global 2rank_gloo; do tail -1 gpurun_out/bench_${TAG}_$f.log | cut -c1-300; done
fi
tail -3 gpurun_out/gpu_tests_$TAG.log; tail -1 gpurun_out/bench_$TAG.log | cut -c1-600
tail -1 gpurun_out/bench_${TAG}_config4_mixed_decode.log | cut -c1-400
exit $rc
