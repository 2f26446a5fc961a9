#!/bin/bash
# Round-4 pass: the deferred-Huffman tests first, then every GPU test, then the default bench line
# (no side legs) -- each step time-limited, chained so the first failure ends the call.
TAG=${1:-r04}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hufjob.py -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/gpu_hufjob_$TAG.log 2>&1 \
&& timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 \
&& timeout -k 10 300 python3 -u bench.py --no-side --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_hufjob_$TAG.log; tail -4 gpurun_out/gpu_tests_$TAG.log; tail -1 gpurun_out/bench_$TAG.log | cut -c1-600
exit $rc
