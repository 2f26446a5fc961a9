#!/bin/bash
# Per-kernel average durations of each library build under ab/*.so (run via gpurun): one rocprofv3
# kernel-trace of a short default bench per build.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abk
for v in ab/*.so; do
  n=$(basename $v .so)
  PGN_LIB=$PWD/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/$n -o run -- \
      python3 bench.py --no-cpu-baseline --no-side --steps 2 --warmup 1 > gpurun_out/abk/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abk/$n.log; exit 1; }
  python3 - "$n" <<'PY'
import csv, glob, sys
n = sys.argv[1]
for f in glob.glob(f"gpurun_out/abk/{n}/**/*kernel_stats.csv", recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if "pgn::" in r["Name"] and "synth" not in r["Name"]]
    print(n, " | ".join(f'{r["Name"].split("(")[0].replace("pgn::", "")} {int(r["Calls"])}x{float(r["AverageNs"]) / 1e6:.3f}ms' for r in rows))
PY
  echo "$n bench $(tail -1 gpurun_out/abk/$n.log | cut -c1-40) $(grep -o '"encode_ms": [0-9.]*, "decode_ms": [0-9.]*' gpurun_out/abk/$n.log)"
done
