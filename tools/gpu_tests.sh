#!/bin/bash
# GPU parity tests only (run via gpurun): tools/gpu_tests.sh TAG [pytest args...]
TAG=${1:-latest}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_tests_$TAG.log
exit $rc
