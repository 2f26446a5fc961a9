#!/bin/bash
# Diagnostic builds of dec_huf_kernel (wrong output, timing only): _ab/libA.so = the product,
# _ab/libD{1,2,3}.so = PGN_K2_DIAG 1 (stores to a junk line), 2 (loads of one block), 3 (no table read).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT/rawnanoporesignalcompression_amd"
make _build/libpgnano_hip.so _build/pgn_pod5file.o >/dev/null
mkdir -p "$ROOT/_ab"
cp _build/libpgnano_hip.so "$ROOT/_ab/libA.so"
for d in ${DIAGS:-1 2 3}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DPGN_K2_DIAG=$d -shared \
      -o "$ROOT/_ab/libD$d.so" csrc/pgn_kernels.hip csrc/pgn_pod5.hip -Wl,_build/pgn_pod5file.o 2>&1 | grep -v "unused during" || true
done
ls -la "$ROOT/_ab"
