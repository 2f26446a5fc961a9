#!/bin/bash
# Multi-block GPU tests first, then the whole GPU suite and a short bench (run via gpurun).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multiblock.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_mb.log 2>&1 || { tail -40 gpurun_out/gpu_mb.log; exit 1; }
tail -12 gpurun_out/gpu_mb.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_mb.log 2>&1 || { tail -40 gpurun_out/gpu_tests_mb.log; exit 1; }
tail -2 gpurun_out/gpu_tests_mb.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-side > gpurun_out/bench_mb.log 2>&1 || exit 1
tail -1 gpurun_out/bench_mb.log | cut -c1-1000
