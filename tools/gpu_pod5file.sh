#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pod5_file.py tests/test_gpu_pod5_batch.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_pod5file.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_pod5file.log
exit $rc
