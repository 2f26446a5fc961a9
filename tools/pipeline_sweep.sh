#!/bin/bash
# Encode/decode time of the bench workload (100,000 x 100,000 samples) over pipeline settings (run via
# gpurun): sub-batch size and resident workgroups per CU of the staged decode, fused vs staged.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 tools/codec_timing.py 100000 3 > gpurun_out/sweep_$name.log 2>&1 || exit 1
  echo "$name ($*): $(tail -1 gpurun_out/sweep_$name.log)"
}
run base
run sb4k PGN_SUBBATCH=4096
run sb16k PGN_SUBBATCH=16384
run sb32k PGN_SUBBATCH=32768
run dwg12 PGN_DEC_WG_PER_CU=12
run ewg12 PGN_ENC_WG_PER_CU=12
run decfused PGN_DEC_PIPELINE=fused
