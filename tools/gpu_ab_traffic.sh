#!/bin/bash
# A/B of _ab/libA.so vs _ab/libB.so (tools/ab_libs.sh): interleaved encode/decode timing, then HBM
# bytes per kernel (FETCH_SIZE, WRITE_SIZE in separate --pmc passes; gfx950 correction 2 x FETCH_SIZE)
# per 100,000-sample chunk.  bash tools/gpu_ab_traffic.sh TAG [READS]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-abt}; R=${2:-20000}
O=gpurun_out/abt_$TAG
mkdir -p $O
for i in 1 2; do
  for L in ${LIBS:-A B}; do
    PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 150 python3 -u tools/codec_timing.py 30000 4 > $O/time_$L$i.log 2>&1 || { tail -3 $O/time_$L$i.log; exit 1; }
    echo "$L$i: $(tail -1 $O/time_$L$i.log)"
  done
done
for L in ${LIBS:-A B}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    PGN_LIB=$PWD/_ab/lib$L.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv \
        -d $O/${L}_$C -o run -- python3 tools/codec_timing.py $R 1 > $O/${L}_$C.log 2>&1 || { echo "$L $C failed"; tail -5 $O/${L}_$C.log; exit 1; }
  done
done
python3 - "$R" "$O" ${LIBS:-A B} <<'PY' | tee $O/summary.txt
import csv, glob, sys, collections
R, O, libs = int(sys.argv[1]), sys.argv[2], sys.argv[3:]
for L in libs:
    v = collections.defaultdict(lambda: collections.defaultdict(float))
    for C in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"{O}/{L}_{C}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].split("::")[-1]
                if r["Kernel_Name"].startswith("pgn::") or "pgn::" in r["Kernel_Name"][:40]:
                    v[k][C] += float(r["Counter_Value"])
    # codec_timing runs K + 1 = 2 encode+decode rounds
    for k, d in sorted(v.items()):
        fetch = 2 * d["FETCH_SIZE"] * 1024 / (2 * R)
        write = d["WRITE_SIZE"] * 1024 / (2 * R)
        print(f"{L} {k:28s} per chunk: read {fetch/1e3:8.1f} KB  write {write/1e3:8.1f} KB  total {(fetch+write)/1e3:8.1f} KB")
PY
