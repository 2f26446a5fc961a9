#!/bin/bash
# A/B of the pipelines (run via gpurun): GPU parity tests, then encode/decode timing of the fused and
# staged pipelines on 30,000 x 100,000-sample reads, then the default bench line.
TAG=${1:-ab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for P in fused staged; do
  PGN_ENC_PIPELINE=$P PGN_DEC_PIPELINE=$P timeout -k 10 120 python3 tools/codec_timing.py 30000 3 > gpurun_out/timing_${TAG}_$P.log 2>&1 || exit 1
  echo "$P: $(tail -1 gpurun_out/timing_${TAG}_$P.log)"
done
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/bench_$TAG.log
