"""The encoder's no-match certificate (pgn_zenc.h no_match_certificate, host restatement
z1m_no_match_certificate): whenever it holds, libzstd 1.4.x's level-1 search (the bytes the GPU
encoder reproduces, zstd1_model.h fast_search_serial) finds no match, so skipping the hash table
cannot change a frame.  Checked against the serial search on the bench's C5 streams and on inputs
built to have matches at every distance."""
import ctypes as C

import numpy as np

import _oracle as O


def _lib():
    m = O.model()
    m.z1m_no_match_certificate.restype = C.c_int
    m.z1m_no_match_certificate.argtypes = [C.c_void_p, C.c_size_t]
    return m


def _nseq(m, a):
    out = np.zeros(3 * max(a.size, 16), np.uint32)
    return m.z1m_sequences(a.ctypes.data_as(C.c_void_p), C.c_size_t(a.size), out.ctypes.data_as(C.c_void_p),
                           C.c_size_t(a.size)) if a.size >= 7 else 0


def _check(m, a):
    a = np.ascontiguousarray(a, np.uint8)
    cert = m.z1m_no_match_certificate(a.ctypes.data_as(C.c_void_p), C.c_size_t(a.size))
    if cert:
        assert _nseq(m, a) == 0
    return cert


def test_certificate_implies_no_sequences_on_c5_streams():
    m = _lib()
    passed = {k: 0 for k in range(5)}
    for r in range(60):
        x = O.synth_read(r, 100_000)
        for k, s in enumerate(O.c5_streams(x)):
            passed[k] += _check(m, np.frombuffer(s, np.uint8))
    # the noise streams (S, M, Llow) are certified almost always
    assert passed[1] >= 55 and passed[2] >= 55


def test_certificate_never_passes_a_block_with_matches():
    m = _lib()
    rng = np.random.default_rng(3)
    for t in range(400):
        n = int(rng.integers(7, 131_073))
        kind = t % 5
        if kind == 0:    # uniform bytes: no matches, certificate expected
            a = rng.integers(0, 256, n)
        elif kind == 1:  # low-entropy bytes: chance matches
            a = rng.integers(0, int(rng.integers(2, 12)), n)
        elif kind == 2:  # a copy of an earlier stretch at a random distance
            a = rng.integers(0, 256, n)
            if n > 64:
                L = int(rng.integers(8, min(4096, n // 2)))
                s0 = int(rng.integers(0, n - 2 * L)) if n > 2 * L else 0
                d0 = int(rng.integers(s0 + L, n - L + 1)) if n - L + 1 > s0 + L else s0 + L
                a[d0:d0 + L] = a[s0:s0 + L]
        elif kind == 3:  # runs (repcode hits)
            a = np.repeat(rng.integers(0, 256, n // 7 + 1), 7)[:n]
        else:            # skewed noise, like the C5 M stream
            a = np.clip(np.abs(rng.normal(0, 40, n)), 0, 255)
        _check(m, a.astype(np.uint8))
