#!/bin/bash
# Full GPU test suite, then encode/decode timing (30,000 reads): bash tools/gpu_check.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-c}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$tag.log
timeout -k 10 200 python3 -u tools/codec_timing.py 30000 5 > gpurun_out/timing_$tag.log 2>&1 || { tail -5 gpurun_out/timing_$tag.log; exit 1; }
tail -1 gpurun_out/timing_$tag.log
