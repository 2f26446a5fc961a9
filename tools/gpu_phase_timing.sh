#!/bin/bash
# encode/decode timing (30,000 reads) then the phase profile (20,000): bash tools/gpu_phase_timing.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-p}
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/codec_timing.py 30000 5 > gpurun_out/timing_$tag.log 2>&1 || { tail -5 gpurun_out/timing_$tag.log; exit 1; }
tail -1 gpurun_out/timing_$tag.log
timeout -k 10 200 python -u tools/phase_profile.py 20000 > gpurun_out/phase_$tag.log 2>&1 || { tail -5 gpurun_out/phase_$tag.log; exit 1; }
sed -n '/^decode:/,/^decode counters/p' gpurun_out/phase_$tag.log
