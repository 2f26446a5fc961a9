#!/bin/bash
# GPU parity tests on the current build, then an interleaved A/B of ab/libA.so vs the current build
# (run via gpurun): tools/gpu_abtest.sh TAG
TAG=${1:-ab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh "PGN_LIB=ab/libA.so" "PGN_LIB=ab/libB.so"
