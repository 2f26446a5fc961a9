#!/bin/bash
# Parity tests + bench (no CPU leg) + per-kernel HBM traffic (run via gpurun): tools/perf_run.sh TAG
TAG=${1:-latest}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 \
&& timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 \
&& bash tools/traffic.sh $TAG > /dev/null 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log; tail -1 gpurun_out/bench_$TAG.log
python3 -c "
import json,sys
d=json.load(open('gpurun_out/traffic_$TAG.json'))
for k,v in d['kernels'].items(): print(k, 'fetch_raw %.2f GB write %.2f GB' % (v['fetch_raw']/1e9, v['write']/1e9))
" 2>/dev/null
exit $rc
