#!/bin/bash
# Build a diagnostic variant of the product library from the working tree with extra compile-time
# definitions: tools/ab_defs.sh NAME "-DPGN_SERIAL_DECODE -DPGN_PROFILE"  ->  _ab/libNAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
T=/tmp/pgn_defs_$N
rm -rf $T && mkdir -p $T && cp -r "$ROOT/rawnanoporesignalcompression_amd" "$ROOT/include" $T/
rm -rf $T/rawnanoporesignalcompression_amd/_build/libpgnano_hip.so
make -C $T/rawnanoporesignalcompression_amd _build/libpgnano_hip.so \
    HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function $*" >/dev/null
mkdir -p "$ROOT/_ab" && cp $T/rawnanoporesignalcompression_amd/_build/libpgnano_hip.so "$ROOT/_ab/lib$N.so"
echo "built _ab/lib$N.so ($*)"
