#!/bin/bash
# Bench-size decode / encode times of one library under several environment settings (run via gpurun):
#   VALS="PGN_DEC_BUFS=2 PGN_DEC_BUFS=3,PGN_HUF_STREAMS=2" bash tools/gpu_env_sweep.sh TAG [LIB]
# (each word of VALS is one setting: comma-separated assignments; "-" = none)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-sweep}
LIB=${2:-$PWD/rawnanoporesignalcompression_amd/_build/libpgnano_hip.so}
O=gpurun_out/$TAG
mkdir -p $O
for i in 1 2; do
  for v in $VALS; do
    a=${v//,/ }
    [ "$a" = "-" ] && a=""
    n=${v//[=,]/_}
    env $a PGN_LIB=$LIB timeout -k 10 200 python3 -u tools/codec_timing.py ${READS:-100000} 3 > $O/$n.$i.log 2>&1 || { tail -3 $O/$n.$i.log; exit 1; }
    echo "$v ($i): $(tail -1 $O/$n.$i.log)"
  done
done
