#!/bin/bash
# Does the merge gain when the intermediate it reads is still in the 256 MB MALL?  Kernel traces of the
# bench-size decode (100,000 chunks) at decode pass sizes PGN_DEFER_G: with 1,024 chunks a pass's
# intermediate (~110 MB touched) is read back while still cached, with 12,500 (default) it is not.
# Serial build (_ab/libSER.so: every decode kernel on one stream, so per-kernel sums are isolated
# times) and the product library (decode wall).  PGN_SUBBATCH lowers the minimum pass size (8,192).  Outputs under gpurun_out/$TAG/.
TAG=${1:-r05_mall}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
rm -rf $O && mkdir -p $O
for lib in SER prod; do
  L=$PWD/_ab/libSER.so; [ $lib = prod ] && L=$PWD/rawnanoporesignalcompression_amd/_build/libpgnano_hip.so
  for G in 1024 2048 4096 12500; do
    PGN_SUBBATCH=$((G < 8192 ? G : 8192)) PGN_DEFER_G=$G PGN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/${lib}_$G -o run -- \
        python3 tools/codec_timing.py 100000 1 > $O/${lib}_$G.log 2>&1 || { tail -5 $O/${lib}_$G.log; exit 1; }
    echo "== $lib PGN_DEFER_G=$G"
    python3 tools/decode_wall.py $O/${lib}_$G/run_kernel_trace.csv 100000 | tail -2
  done
done
