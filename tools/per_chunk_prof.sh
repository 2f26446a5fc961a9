#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/per_chunk_probe.py 200 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pc -o run -- python3 tools/per_chunk_probe.py 200 > gpurun_out/prof_pc.log 2>&1
rc=$?
cat gpurun_out/prof_pc/run_kernel_stats.csv 2>/dev/null | cut -c1-160 | head -12
exit $rc
