#!/bin/bash
# Build a variant library from the working tree with a sed expression applied to the kernel sources:
# tools/ab_variant.sh NAME 'sed-expr'  ->  _ab/libNAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
T=/tmp/pgn_var_$N
rm -rf $T && mkdir -p $T && cp -r "$ROOT/rawnanoporesignalcompression_amd" "$ROOT/include" $T/
sed -i "$1" $T/rawnanoporesignalcompression_amd/csrc/pgn_kernels.hip
make -C $T/rawnanoporesignalcompression_amd _build/libpgnano_hip.so >/dev/null
mkdir -p "$ROOT/_ab" && cp $T/rawnanoporesignalcompression_amd/_build/libpgnano_hip.so "$ROOT/_ab/lib$N.so"
echo "built _ab/lib$N.so"
