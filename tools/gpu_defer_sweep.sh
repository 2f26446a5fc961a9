#!/bin/bash
# Bench step time for decode pass sizes (PGN_DEFER_G): bash tools/gpu_defer_sweep.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-ds}
mkdir -p gpurun_out
for G in ${GS:-16384 25000 32768 50000}; do
  PGN_DEFER_G=$G timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/defer_${TAG}_$G.log 2>&1 || { tail -5 gpurun_out/defer_${TAG}_$G.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/defer_${TAG}_$G.log').read().strip().splitlines()[-1]); print('G=$G', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'])"
done
