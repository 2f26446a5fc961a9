#!/bin/bash
# pod5 batch GPU tests first, then the whole GPU suite (run via gpurun).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pod5_batch.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_pod5.log 2>&1 || { tail -40 gpurun_out/gpu_pod5.log; exit 1; }
tail -8 gpurun_out/gpu_pod5.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_pod5.log 2>&1 || { tail -40 gpurun_out/gpu_tests_pod5.log; exit 1; }
tail -2 gpurun_out/gpu_tests_pod5.log
