#!/bin/bash
# Phase-cycle profile of encode/decode (run via gpurun): tools/phase_run.sh TAG [READS]
TAG=${1:-latest}
R=${2:-20000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/phase_profile.py $R > gpurun_out/phase_$TAG.log 2>&1
rc=$?
tail -40 gpurun_out/phase_$TAG.log
exit $rc
