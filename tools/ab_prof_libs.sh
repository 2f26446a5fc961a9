#!/bin/bash
# Phase-profile builds (-DPGN_PROFILE) of git HEAD (or $1) and the working tree: _ab/libA_prof.so, _ab/libB_prof.so
set -e
REF=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf /tmp/pgn_ab_base && git -C "$ROOT" worktree add -f --detach /tmp/pgn_ab_base "$REF" >/dev/null 2>&1
make -C /tmp/pgn_ab_base/rawnanoporesignalcompression_amd _build/libpgnano_hip_prof.so >/dev/null
mkdir -p "$ROOT/_ab"
cp /tmp/pgn_ab_base/rawnanoporesignalcompression_amd/_build/libpgnano_hip_prof.so "$ROOT/_ab/libA_prof.so"
git -C "$ROOT" worktree remove --force /tmp/pgn_ab_base
make -C "$ROOT/rawnanoporesignalcompression_amd" _build/libpgnano_hip_prof.so >/dev/null
cp "$ROOT/rawnanoporesignalcompression_amd/_build/libpgnano_hip_prof.so" "$ROOT/_ab/libB_prof.so"
echo "built _ab/libA_prof.so ($REF) and _ab/libB_prof.so (working tree)"
