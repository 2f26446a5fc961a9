"""CPU baseline check (build container, one thread): the oracle's C5 encode / decode (oracle/pgn_oracle.c,
a C restatement of C5.hpp:282-683 over libzstd) against the reference's own compiled split / merge
(oracle/_ref libpgn_ref.so: C5.hpp:57-257 built verbatim) plus the same five ZSTD_compress /
ZSTD_decompress calls on the same libzstd, on the bench's synthetic reads.

    python3 tools/oracle_vs_ref_timing.py [reads] [samples]

The reference leg leaves out what cannot be built here: its ten Arrow buffer allocations per encoded
chunk (C5.hpp:293-297, pgnano.cpp:66-68) and the frame assembly copies (C5.hpp:429-462).  So it is a
lower bound on the reference's own time, and oracle/reference > 1 means the oracle is faster than the
reference would be.  Needs /root/reference (the reference library is built from it).
"""
import ctypes as C
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import _oracle as O  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
    L, ref = O.oracle(), O.ref()
    if ref is None:
        sys.exit("reference sources absent: nothing to compare")
    Z = C.CDLL(L.pgno_zstd_path().decode())
    Z.ZSTD_compress.restype = C.c_size_t
    Z.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
    Z.ZSTD_decompress.restype = C.c_size_t
    Z.ZSTD_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
    Z.ZSTD_compressBound.restype = C.c_size_t
    reads = [O.synth_read(r, n) for r in range(R)]
    cap = int(L.pgno_c5_bound(n))
    blob = np.zeros(cap + 64, np.uint8)
    out = np.zeros(n, np.int16)
    olen = C.c_size_t()
    # oracle
    blobs = []
    t = time.perf_counter()
    for x in reads:
        rc = L.pgno_c5_compress(x.ctypes.data, n, blob.ctypes.data, cap, C.byref(olen), None)
        assert rc == 0
        blobs.append(blob[:olen.value].copy())
    t_oe = time.perf_counter() - t
    t = time.perf_counter()
    for b, x in zip(blobs, reads):
        assert L.pgno_c5_decompress(b.ctypes.data, b.size, out.ctypes.data, n) == 0
    t_od = time.perf_counter() - t
    # reference split / merge + the same libzstd calls
    sbuf = np.zeros(5 * (n + 64) + 3 * n + 64, np.uint8)
    offs, sz = np.zeros(5, np.uint64), np.zeros(5, np.uint64)
    fb = int(Z.ZSTD_compressBound(n))
    frames = [np.zeros(fb + 64, np.uint8) for _ in range(5)]
    inter = np.zeros(5 * n + 64, np.uint8)
    rec = []
    t = time.perf_counter()
    for x in reads:
        assert ref.pgnr_encode(0, x.ctypes.data, n, sbuf.ctypes.data, offs.ctypes.data, sz.ctypes.data) == 5
        fl = []
        for s in range(5):
            r = Z.ZSTD_compress(frames[s].ctypes.data, fb, sbuf.ctypes.data + int(offs[s]), int(sz[s]), 1)
            fl.append(r)
        rec.append(([frames[s][:fl[s]].copy() for s in range(5)], [int(v) for v in sz]))
    t_re = time.perf_counter() - t
    d = np.zeros(5, np.uint64)
    t = time.perf_counter()
    for fr, szs in rec:
        off = 0
        for s in range(5):
            r = Z.ZSTD_decompress(inter.ctypes.data + off, szs[s], fr[s].ctypes.data, fr[s].size)
            assert r == szs[s]
            d[s] = r
            off += r
        ref.pgnr_decode(0, inter.ctypes.data, off, d.ctypes.data, out.ctypes.data, n)
    t_rd = time.perf_counter() - t
    S = R * n / 1e6
    print(f"{R} reads x {n} samples, one thread, libzstd {L.pgno_zstd_version()} ({L.pgno_zstd_path().decode()})")
    print(f"oracle    encode {S / t_oe:8.1f} MS/s  decode {S / t_od:8.1f} MS/s")
    print(f"reference encode {S / t_re:8.1f} MS/s  decode {S / t_rd:8.1f} MS/s  (split/merge built from C5.hpp, "
          "no Arrow allocations or assembly copies)")
    print(f"oracle / reference: encode {t_re / t_oe:.3f}  decode {t_rd / t_od:.3f}")


if __name__ == "__main__":
    main()
