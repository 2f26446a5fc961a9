#!/bin/bash
# Round-4 evidence (second session): the evidence pass of tools/gpu_r04g.sh, then an interleaved A/B
# of _ab/libA.so / libB.so at 30,000 chunks.
TAG=${1:-r04b}
bash tools/gpu_r04g.sh $TAG || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2; do
  for L in A B; do
    echo "$L$i: $(PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 120 python3 -u tools/codec_timing.py 30000 4 2>&1 | tail -1)"
  done
done | tee gpurun_out/ab_${TAG}.log
