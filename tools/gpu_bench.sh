#!/bin/bash
# bench.py (no CPU leg, no side legs) on the GPU box: bash tools/gpu_bench.sh TAG [extra bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-b}; shift
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-side "$@" > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log | cut -c1-1500
