#!/bin/bash
# GPU tests, then the per-chunk plugin probe (200 calls each way): bash tools/gpu_pc.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-pc}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
for i in 1 2; do timeout -k 10 120 python3 tools/per_chunk_probe.py 300 || exit 1; done
