#!/bin/bash
# per-chunk plugin call latency under each encode pipeline (run via gpurun)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for P in fused staged; do
  echo "$P: $(PGN_ENC_PIPELINE=$P timeout -k 10 120 python3 tools/per_chunk_probe.py 200 2>/dev/null | tail -1)" || exit 1
done
