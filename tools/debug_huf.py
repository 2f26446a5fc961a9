"""Diagnostic: decode one synthetic chunk with the printf build (_build/libpgnano_hip_dbg.so)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np

from rawnanoporesignalcompression_amd import _native

_native._lib = _native.load(os.path.join(os.path.dirname(_native.LIB_PATH), "libpgnano_hip_dbg.so"))
import _oracle as O
from rawnanoporesignalcompression_amd import PGNanoCodec

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
x = O.synth_read(3, n)
rc, blob, _ = O.c5_compress(x)
c = PGNanoCodec(0)
try:
    y = c.decompress_signal(blob, sample_count=n)
    print("decode ok", np.array_equal(x, y))
except Exception as e:
    print("decode failed:", e)
import ctypes as C
L = _native.load()
buf = np.zeros(1 + (1 << 18), np.uint32)
L.pgn_debug_huf_dump.argtypes = [C.c_void_p, C.c_size_t]
L.pgn_debug_huf_dump(buf.ctypes.data, buf.size)
cnt = int(buf[0])
rec = buf[1:1 + min(cnt, 1 << 18)].reshape(-1, 8).astype(np.int64)
rec = np.where(rec >= 2**31, rec - 2**32, rec)
print("records", len(rec))
for r in rec[:4000]:
    t = int(r[0])
    if t == 1:
        print("start k=%d j=%d T=%d sl=%d nsym=%d tl=%d rs=%d" % tuple(r[1:8]))
    elif t == 3:
        print("end   k=%d j=%d T=%d produced=%d nsym=%d" % tuple(r[1:6]))
    else:
        k, j = (t - 2) % 256 // 16, (t - 2) // 256
        cx = int(r[7]) & 0xFFFFFFFF
        ex = cx >> 16
        ex = ex - 65536 if ex >= 32768 else ex
        print("round k=%d j=%2d T=%d hi=%d lo=%d c=%d q=%d entry=%d cnt=%d ex=%d" % (k, j, r[1], r[2], r[3], r[4], r[5], r[6], cx & 0xFFFF, ex))
