"""The oracle's split/merge pinned against the reference's OWN svb16 code.

oracle/ref.mk compiles the `namespace svb16` block of every pgnano variant header (C5.hpp:27-277,
C4.hpp:27-269, C3.hpp:27-208, C2.hpp:27-191, C1.hpp:31-197, VBZ_0.hpp:30-311) verbatim from
/root/reference, plus the pod5 VBZ codec's svb16 stage (pod5_format/svb16/encode.hpp, decode.hpp),
into oracle/_ref/.  Here oracle/pgn_oracle.c must produce exactly the streams those functions produce
(the bytes each variant hands to ZSTD_compress) and exactly their decoded samples and consumed counts
(the value behind "Remaining data at end of signal buffer"), on the reference's own POD5 fixture, the
threshold sizes, stress signals and a random fuzz.

Where /root/reference is absent (the GPU box) these tests skip; tests/golden/c5_golden.json then
carries the reference-produced stream digests (`ref_streams_sha256`, written by make_golden.py from
the compiled reference) and test_golden_ref_stream_digests checks the oracle against them.
"""
import hashlib

import numpy as np
import pytest

import _oracle as O
from _golden import golden, real_vbz_chunks

VARIANTS = list(O.VARIANTS)
EDGE = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 33, 63, 64, 65, 255, 256, 257, 1023, 1024, 1025, 16384, 16385,
        65791, 65792, 65793, 102399, 102400, 131072, 200000]

# decided from the reference tree alone, so that a process without it (the GPU box) never loads the
# libraries built from it
needs_ref = pytest.mark.skipif(not O.ref_available(), reason="reference sources not present (/root/reference)")


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _real_signals():
    out = []
    for vbz, n in real_vbz_chunks():
        rc, x = O.vbz_decompress(vbz, n)
        assert rc == 0
        out.append(x)
    return out


def _deltas_signal(rng, n, weights):
    """A signal whose zig-zag deltas fall in the chosen class ranges (0 / 1-16 / 17-272 / 273+)."""
    cls = rng.choice(4, size=n, p=weights)
    v = np.where(cls == 0, 0,
                 np.where(cls == 1, rng.integers(1, 17, n),
                          np.where(cls == 2, rng.integers(17, 273, n), rng.integers(273, 65536, n))))
    # zig-zag decode: d = (v >> 1) ^ -(v & 1), then cumulative sum mod 2^16
    d = ((v >> 1) ^ -(v & 1)).astype(np.int64)
    return (np.cumsum(d) & 0xFFFF).astype(np.uint16).view(np.int16)


def _stress_signals():
    rng = np.random.default_rng(1234)
    s = {
        "constant": np.full(5000, 517, np.int16),
        "alternating_extremes": np.tile(np.array([32767, -32768], np.int16), 2500),
        "extremes_mix": rng.choice(np.array([32767, -32768, 0, -1, 1], np.int16), 7001),
        "uniform_int16": rng.integers(-32768, 32768, 9999).astype(np.int16),
        "ramp": (np.arange(70000) * 7).astype(np.int16),
        "class_boundaries": _deltas_signal(rng, 4097, [0.25, 0.25, 0.25, 0.25]),
        "all_small": _deltas_signal(rng, 3001, [0.0, 1.0, 0.0, 0.0]),
        "all_medium": _deltas_signal(rng, 3002, [0.0, 0.0, 1.0, 0.0]),
        "all_large": _deltas_signal(rng, 3003, [0.0, 0.0, 0.0, 1.0]),
        "odd_nibbles": _deltas_signal(rng, 4099, [0.1, 0.6, 0.25, 0.05]),
    }
    # exact class thresholds of C5 (v = 0, 1, 16, 17, 272, 273, 65535) and of C4 (15, 16, 255, 256)
    v = np.array([0, 1, 16, 17, 272, 273, 65535, 15, 255, 256, 2, 18, 274] * 37)
    d = ((v >> 1) ^ -(v & 1)).astype(np.int64)
    s["thresholds"] = (np.cumsum(d) & 0xFFFF).astype(np.uint16).view(np.int16)
    return s


def _check_split(variant, x):
    ref = O.ref_variant_streams(variant, x)
    ours = O.variant_streams(variant, x)
    assert len(ref) == len(ours), variant
    for s, (a, b) in enumerate(zip(ref, ours)):
        assert a == b, f"{variant} stream {s} differs (n={x.size}): {len(a)} vs {len(b)} bytes"
    return ref


def _check_merge(variant, x, streams, rng=None):
    inter = b"".join(streams)
    d = [len(s) for s in streams]
    out_r, cons_r = O.ref_variant_merge(variant, inter, d, x.size)
    rc, out_o, cons_o = O.oracle_variant_merge(variant, inter, d, x.size)
    assert rc == O.OK
    assert np.array_equal(out_r, x) and np.array_equal(out_o, x), variant
    assert cons_r == cons_o, (variant, cons_r, cons_o)
    if rng is None or x.size == 0:
        return
    # perturbed stream sizes (the pointer walk reads across stream borders) and trailing bytes
    # (consumed != size: the "Remaining data" case); the buffer is padded so that every read the
    # reference makes stays inside it (the reference does not bounds-check)
    pad = rng.integers(0, 256, 2 * x.size + 64, dtype=np.uint8).tobytes()
    for _ in range(4):
        dd = [max(0, v + int(rng.integers(-3, 4))) for v in d]
        dd[0] = d[0]
        out_r, cons_r = O.ref_variant_merge(variant, inter + pad, dd, x.size)
        rc, out_o, cons_o = O.oracle_variant_merge(variant, inter + pad, dd, x.size)
        assert rc == O.OK, (variant, rc)
        assert np.array_equal(out_r, out_o), variant
        assert cons_r == cons_o, (variant, dd, cons_r, cons_o)


@needs_ref
@pytest.mark.parametrize("variant", VARIANTS)
def test_reference_fixture_split_and_merge(variant):
    """All 22 chunks of pod5/test_data/multi_fast5_zip_v3.pod5 (the reference's own fixture)."""
    rng = np.random.default_rng(7)
    for x in _real_signals():
        st = _check_split(variant, x)
        _check_merge(variant, x, st, rng)


@needs_ref
@pytest.mark.parametrize("variant", VARIANTS)
def test_edge_sizes(variant):
    rng = np.random.default_rng(11)
    for n in EDGE:
        x = O.synth_read(1000 + n, n)
        st = _check_split(variant, x)
        _check_merge(variant, x, st, rng if n <= 20000 else None)


@needs_ref
@pytest.mark.parametrize("variant", VARIANTS)
def test_stress_signals(variant):
    rng = np.random.default_rng(13)
    for name, x in _stress_signals().items():
        st = _check_split(variant, x)
        _check_merge(variant, x, st, rng)


@needs_ref
@pytest.mark.parametrize("variant", VARIANTS)
def test_fuzz(variant):
    rng = np.random.default_rng(100 + O.VARIANTS[variant])
    for it in range(150):
        n = int(rng.integers(0, 3000)) if it % 10 else int(rng.integers(3000, 40000))
        w = rng.dirichlet(np.ones(4) * 0.7)
        x = _deltas_signal(rng, n, w)
        st = _check_split(variant, x)
        _check_merge(variant, x, st, rng)


@needs_ref
def test_c5_class_counters_match_reference():
    """number_small / number_medium / number_large (C5.hpp:110-139) equal the class counts in our keys."""
    O.ref_counters(reset=True)
    tot = np.zeros(4, np.int64)
    for x in _real_signals()[:6]:
        O.ref_variant_streams("C5", x)
        keys = np.frombuffer(O.variant_streams("C5", x)[0], np.uint8)
        codes = ((keys[:, None] >> (2 * np.arange(4))) & 3).reshape(-1)[: x.size]
        tot += np.bincount(codes, minlength=4)
    c = O.ref_counters(reset=True)
    assert (c["small"], c["medium"], c["large"]) == (int(tot[1]), int(tot[2]), int(tot[3]))


@needs_ref
def test_vbz_svb16_stage_matches_reference():
    """pod5 VBZ svb16 stage (signal_compression.cpp:49-50, 134-135), SSE4.1 decode as the reference builds."""
    rng = np.random.default_rng(3)
    signals = _real_signals() + list(_stress_signals().values())
    signals += [O.synth_read(2000 + n, n) for n in EDGE if n <= 131072]
    for x in signals:
        a = O.ref_vbz_svb_encode(x)
        assert a == O.oracle_vbz_svb_encode(x)
        back, consumed = O.ref_vbz_svb_decode(a, x.size)
        assert np.array_equal(back, x) and consumed == len(a)
    del rng


def test_golden_ref_stream_digests():
    """Runs without the reference tree: the oracle's C5 streams on the fixture equal the digests the
    compiled reference produced when tests/golden/make_golden.py was run."""
    g = golden()
    assert g.get("ref_pinned", {}).get("c5_streams"), "c5_golden.json lacks the reference check"
    for x, meta in zip(_real_signals(), g["real"]):
        got = [sha(s) for s in O.variant_streams("C5", x)]
        assert got == meta["ref_streams_sha256"]
