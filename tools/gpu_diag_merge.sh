#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PGN_LIB=$PWD/_ab/libM.so timeout -k 10 120 python3 -u tools/codec_timing.py 30000 5 > gpurun_out/dm_full.log 2>&1; echo "full: $(tail -1 gpurun_out/dm_full.log)"
PGN_DIAG_SKIP_MERGE=1 PGN_LIB=$PWD/_ab/libM.so timeout -k 10 120 python3 -u tools/codec_timing.py 30000 5 > gpurun_out/dm_skip.log 2>&1; echo "skip merge: $(tail -1 gpurun_out/dm_skip.log)"
