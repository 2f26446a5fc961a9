#!/bin/bash
# A/B of library builds under ab/*.so (run via gpurun): decode-only and full bench lines per variant,
# interleaved twice.  tools/ab_decode.sh [bench args...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ab/*.so; do
    PGN_LIB=$PWD/$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-side --steps 3 "$@" > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$v rep$rep $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("enc", d["encode_ms"], "dec", d["decode_ms"], "ok", d["round_trip_ok"])')"
  done
done
