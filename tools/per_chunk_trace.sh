#!/bin/bash
# Kernel + memory-copy + HIP API trace of the per-chunk probe (no counters), then its timeline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
    -d gpurun_out/pc_trace -o run -- python3 tools/per_chunk_probe.py 100 > gpurun_out/pc_trace.log 2>&1 \
&& python3 tools/per_chunk_timeline.py gpurun_out/pc_trace > gpurun_out/pc_timeline.txt
rc=$?
head -80 gpurun_out/pc_timeline.txt
exit $rc
