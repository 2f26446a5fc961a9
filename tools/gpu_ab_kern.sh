#!/bin/bash
# Interleaved A/B of library builds (run via gpurun): bench-size encode / decode times (100,000 chunks,
# several decode passes) and, from a kernel trace of a 20,000-chunk call (one decode pass: every decode
# kernel in order on one stream), each kernel's own duration.  LIBS="A B C" picks _ab/lib*.so.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-abk}
O=gpurun_out/$TAG
mkdir -p $O
for L in ${LIBS:-A B}; do
  PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/k_$L -o run -- \
      python3 tools/codec_timing.py 20000 1 > $O/k_$L.log 2>&1 || { tail -3 $O/k_$L.log; exit 1; }
  echo "$L kernels (20,000 chunks): $(python3 tools/decode_wall.py $O/k_$L/run_kernel_trace.csv | tail -1 | cut -d: -f2-)"
done
for i in 1 2; do
  for L in ${LIBS:-A B}; do
    PGN_LIB=$PWD/_ab/lib$L.so timeout -k 10 200 python3 -u tools/codec_timing.py 100000 3 > $O/t_$L$i.log 2>&1 || { tail -3 $O/t_$L$i.log; exit 1; }
    echo "$L$i: $(tail -1 $O/t_$L$i.log)"
  done
done
