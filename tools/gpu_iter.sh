#!/bin/bash
# One iteration: the decode/encode GPU parity subset on the in-tree library, then A/B timing and
# per-kernel HBM bytes of _ab/libA.so vs _ab/libB.so.  bash tools/gpu_iter.sh TAG [TESTS...]
TAG=${1:-it}; shift
TESTS=${*:-tests/test_gpu_parity.py tests/test_gpu_hufjob.py tests/test_gpu_cross_stream.py tests/test_gpu_multiblock.py}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > gpurun_out/iter_tests_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/iter_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/iter_tests_$TAG.log
bash tools/gpu_ab_traffic.sh $TAG 20000
