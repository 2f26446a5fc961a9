#!/bin/bash
# POD5 host batch path: copy-worker and sub-batch sweep (run via gpurun)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for T in 4 8 16; do for M in 16 64; do
PGN_HOST_THREADS=$T PGN_POD5_SUBBATCH_MB=$M timeout -k 10 120 python3 -u - > gpurun_out/host2_${T}_$M.log 2>&1 <<'PY'
import os, sys, json
sys.path.insert(0, os.getcwd())
import torch, bench
from rawnanoporesignalcompression_amd import PGNanoCodec
c = PGNanoCodec(0)
print(json.dumps(bench.pod5_batch_host(torch, c, 100000, 42)))
PY
echo "threads $T sub $M MB: $(tail -1 gpurun_out/host2_${T}_$M.log | cut -c1-120)"
done; done
