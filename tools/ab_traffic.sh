#!/bin/bash
# HBM traffic of the encode kernel per library build _ab/lib$n.so, n in LIBS (run via gpurun): the PGN_AB_SKIP
# diagnostic builds stop the zstd stage after successive phases (1: no zstd stage, raw blocks; 2: match
# search, then raw blocks; 3: + literal gather and histograms, raw literals; 4: + Huffman tables, no bit
# packing; 0: the product), so the differences attribute enc_chunk_kernel's bytes to its phases.
# FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md), gfx950 correction 2 x FETCH_SIZE.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abt
R=${1:-20000}
for n in ${LIBS:-A B}; do
  v=_ab/lib$n.so
  for C in FETCH_SIZE WRITE_SIZE; do
    PGN_ENCODE_ONLY=1 PGN_LIB=$PWD/$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv \
        -d gpurun_out/abt/${n}_$C -o run -- python3 tools/traffic_probe.py $R 100000 \
        > gpurun_out/abt/${n}_$C.log 2>&1 || { echo "$n $C failed"; tail -5 gpurun_out/abt/${n}_$C.log; exit 1; }
  done
done
python3 - "$R" <<'PY' | tee gpurun_out/abt/summary.txt
import csv, glob, sys, collections
R = int(sys.argv[1])
for d in sorted(glob.glob("gpurun_out/abt/*_FETCH_SIZE")):
    n = d.split("/")[-1][:-len("_FETCH_SIZE")]
    v = collections.defaultdict(float)
    for C in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"gpurun_out/abt/{n}_{C}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Kernel_Name"].split("(")[0].split("::")[-1].startswith("enc_chunk_kernel"):
                    v[C] += float(r["Counter_Value"])
    fetch = 2 * v["FETCH_SIZE"] * 1024 / R  # KB units -> bytes, gfx950 correction
    write = v["WRITE_SIZE"] * 1024 / R
    print(f"{n}: enc_chunk_kernel per 100,000-sample chunk: read {fetch/1e3:.1f} KB (raw {fetch/2e3:.1f}), "
          f"write {write/1e3:.1f} KB, total {(fetch+write)/1e3:.1f} KB")
PY
