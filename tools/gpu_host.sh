#!/bin/bash
# POD5 batch / file GPU tests and the host-memory side numbers of bench.py (run via gpurun)
TAG=${1:-h}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pod5_batch.py tests/test_gpu_pod5_file.py tests/test_pod5_signal.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u - > gpurun_out/host_$TAG.log 2>&1 <<'PY'
import os, sys, json, time
sys.path.insert(0, os.getcwd())
import torch, bench
from rawnanoporesignalcompression_amd import PGNanoCodec
c = PGNanoCodec(0)
for i in range(2):
    r = bench.pod5_batch_host(torch, c, 100000, 42)
    print(json.dumps(r))
print(json.dumps(bench.per_chunk_plugin(torch, c, 100000, 42)))
PY
rc=$?; cat gpurun_out/host_$TAG.log | tail -4; exit $rc
