#!/bin/bash
# Build the committed library (git HEAD, or $1) as _ab/libA.so and the working tree's as _ab/libB.so
# (A/B timing on one GPU box: PGN_LIB selects the library).
set -e
REF=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf /tmp/pgn_ab_base && git -C "$ROOT" worktree add -f --detach /tmp/pgn_ab_base "$REF" >/dev/null 2>&1
make -C /tmp/pgn_ab_base/rawnanoporesignalcompression_amd _build/libpgnano_hip.so >/dev/null
mkdir -p "$ROOT/_ab"
cp /tmp/pgn_ab_base/rawnanoporesignalcompression_amd/_build/libpgnano_hip.so "$ROOT/_ab/libA.so"
git -C "$ROOT" worktree remove --force /tmp/pgn_ab_base
make -C "$ROOT/rawnanoporesignalcompression_amd" _build/libpgnano_hip.so >/dev/null
cp "$ROOT/rawnanoporesignalcompression_amd/_build/libpgnano_hip.so" "$ROOT/_ab/libB.so"
echo "built _ab/libA.so ($REF) and _ab/libB.so (working tree)"
