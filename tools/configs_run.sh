#!/bin/bash
# The bench's other BASELINE configs (run via gpurun): configs[2] (R10.4.1 generator, C5 vs VBZ ratio)
# and configs[4] (mixed pores, decode only), after the GPU tests and the default bench line.
TAG=${1:-cfg}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --pore r1041 --compare-vbz --no-cpu-baseline --no-side > gpurun_out/bench_${TAG}_config3.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --mixed-pores --decode-only --no-cpu-baseline --no-side > gpurun_out/bench_${TAG}_config5.log 2>&1 || exit 1
for f in gpurun_out/bench_$TAG.log gpurun_out/bench_${TAG}_config3.log gpurun_out/bench_${TAG}_config5.log; do tail -1 $f | cut -c1-700; done
