#!/bin/bash
# GPU parity tests with the default pipeline choice, then the encode tests with the staged pipeline
# forced for every batch size, then the per-chunk call latency (run via gpurun)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_auto.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_auto.log; [ $rc -eq 0 ] || exit $rc
PGN_ENC_PIPELINE=staged timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiblock.py tests/test_gpu_vbz.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_staged.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_staged.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/per_chunk_probe.py 200 2>/dev/null | tail -1
