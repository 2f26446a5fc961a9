#!/bin/bash
# GPU test suite (optionally a -k filter): bash tools/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
tag=${1:-t}
mkdir -p gpurun_out
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$2" > gpurun_out/gpu_tests_$tag.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1
fi
rc=$?
tail -25 gpurun_out/gpu_tests_$tag.log
exit $rc
