#!/bin/bash
# A/B arms (tools/ab_env.sh) followed by the phase profile of the current build (run via gpurun):
# tools/gpu_ab_phase.sh TAG "ARM1" "ARM2" ...
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_env.sh "$@" && bash tools/phase_run.sh $TAG > /dev/null && grep -A22 "^decode:" gpurun_out/phase_$TAG.log
