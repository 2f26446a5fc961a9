#!/bin/bash
# A/B of environment settings (run via gpurun): tools/ab_env.sh "ENV1" "ENV2" ... ; each arg is a
# space-separated list of VAR=value for one arm (empty string = defaults).  Interleaved twice.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in "$@"; do
    env $arm timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-side --steps 3 > gpurun_out/ab_env.log 2>&1 || { tail -5 gpurun_out/ab_env.log; exit 1; }
    echo "[$arm] rep$rep $(tail -1 gpurun_out/ab_env.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("enc", d["encode_ms"], "dec", d["decode_ms"], "ok", d["round_trip_ok"])')"
  done
done
