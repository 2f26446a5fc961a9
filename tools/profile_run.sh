#!/bin/bash
# Kernel-trace profile of the default bench (run on the GPU box): writes gpurun_out/prof_<tag>/
set -e
TAG=${1:-r01}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --no-side "$@" > gpurun_out/prof_$TAG.bench.log 2>&1
