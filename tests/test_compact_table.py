"""Host restatement of the deferred Huffman job's compact table (pgn_zdec.h job_segments, pgn_hufjob.h),
checked three ways.

The table keeps three segments of the full single-symbol decode table (HUF_readDTableX1: weight w owns
the entries [rankStart[w], rankStart[w] + cnt[w] << (w - 1)), symbols in (weight, symbol) order):
[0, T1) whole, [T1, T2) one entry per 2^d1, [T2, 2^tl) one per 2^d2, with T[d] = the entries whose code
is longer than tl - d bits; (d1, d2) are chosen for the smallest table.  huf_defer_body counts T[d]
from the full table and gathers the entries from it; dec_frame_fast (huf_build_dtable_body with a job
table) computes the same entries from the ranks alone (T[d] = rankStart[d + 1], entry idx belongs to the
last weight whose range starts at or below it).  Both are restated here over random weight sets (every
table log 5..11, skewed and flat) and must agree entry for entry with the same segments; and the
kernel's lookup, compact[min(p, (p >> d1) + C1, (p >> d2) + C2)], must equal full[p] for every peek p.
"""
import numpy as np

K_JOB_TAB_USE = 352


def _full_table(weights, tl):
    """HUF_readDTableX1's table: entry = (symbol, nbBits)"""
    cnt = np.bincount(weights, minlength=13)
    rank_start, before = {}, {}
    nu = no = 0
    for w in range(1, 13):
        rank_start[w], before[w] = nu, no
        if w <= tl:
            nu += int(cnt[w]) << (w - 1)
        no += int(cnt[w])
    order = sorted((w, s) for s, w in enumerate(weights) if w)
    full = [None] * (1 << tl)
    for w in range(1, tl + 1):
        a = rank_start[w]
        for u in range(a, a + (int(cnt[w]) << (w - 1))):
            s = order[before[w] + ((u - a) >> (w - 1))][1]
            full[u] = (s, tl + 1 - w)
    return full, cnt, rank_start, before, order


def _segments(T, tl):
    """pgn_zdec.h job_segments: T[d] for d = 0..7 -> (d1, d2, T1, T2, C1, C2, size)"""
    tsz = 1 << tl
    best = (0, 0, 0, 0, tsz)
    dmax = min(tl - 1, 7)
    for d1 in range(0, 7):
        for d2 in range(d1 + 1, 8):
            if d2 > dmax:
                continue
            t1, t2 = T[d1], T[d2]
            sz = t1 + ((t2 - t1) >> d1) + ((tsz - t2) >> d2)
            if sz < best[4]:
                best = (d1, d2, t1, t2, sz)
    d1, d2, t1, t2, size = best
    c1 = t1 - (t1 >> d1)
    c2 = t1 + ((t2 - t1) >> d1) - (t2 >> d2)
    return d1, d2, t1, t2, c1, c2, size


def _entry_index(sg, j):
    d1, d2, t1, t2, c1, c2, _ = sg
    return j if j < t1 else ((j - c1) << d1 if j < t1 + ((t2 - t1) >> d1) else (j - c2) << d2)


def _compact_from_full(full, tl):
    T = [0] + [sum(1 for e in full if e[1] + d > tl) for d in range(1, 8)]
    sg = _segments(T, tl)
    if sg[6] > K_JOB_TAB_USE:
        return None
    return sg, [full[_entry_index(sg, j)] for j in range(sg[6])]


def _compact_from_ranks(cnt, rank_start, before, order, tl):
    T = [rank_start[d + 1] for d in range(8)]
    sg = _segments(T, tl)
    if sg[6] > K_JOB_TAB_USE:
        return None
    out = []
    for j in range(sg[6]):
        idx = _entry_index(sg, j)
        w = rs0 = bf = 0
        for ww in range(1, 13):
            if ww <= tl and cnt[ww] and rank_start[ww] <= idx:
                w, rs0, bf = ww, rank_start[ww], before[ww]
        out.append((order[bf + ((idx - rs0) >> (w - 1))][1], tl + 1 - w))
    return sg, out


def _random_weights(rng, tl, nsym, skew):
    """Huffman weights (1..tl) of nsym symbols whose table fills exactly 2^tl entries"""
    while True:
        lens = np.clip(np.round(rng.normal(tl - 1 - skew, 1.2 + skew, nsym)), 1, tl).astype(int)
        total = sum(1 << (tl - l) for l in lens)
        while total > (1 << tl):  # lengthen codes until the Kraft sum fits
            i = int(rng.integers(0, nsym))
            if lens[i] < tl:
                total -= 1 << (tl - lens[i] - 1)
                lens[i] += 1
        while total < (1 << tl):  # shorten codes until it is exact
            i = int(rng.integers(0, nsym))
            if lens[i] > 1 and total + (1 << (tl - lens[i])) <= (1 << tl):
                total += 1 << (tl - lens[i])
                lens[i] -= 1
            elif all(l == 1 for l in lens):
                break
        if total == (1 << tl):
            return [tl + 1 - int(l) for l in lens]


def test_compact_table_from_ranks_equals_gather():
    rng = np.random.default_rng(5)
    checked = 0
    for tl in range(5, 12):
        for skew in (0.0, 1.0, 2.5):
            for nsym in (2 ** (tl - 3), 2 ** (tl - 2), min(256, 2 ** (tl - 1))):
                weights = _random_weights(rng, tl, max(nsym, 2), skew)
                full, cnt, rank_start, before, order = _full_table(weights, tl)
                assert all(e is not None for e in full)
                a = _compact_from_full(full, tl)
                b = _compact_from_ranks(cnt, rank_start, before, order, tl)
                assert a == b, (tl, skew, nsym)
                if a is None:
                    continue
                checked += 1
                # the kernel's lookup (dec_huf_kernel): the entry of every peek is the full table's
                (d1, d2, _, _, c1, c2, _), comp = a
                for p in range(1 << tl):
                    assert comp[min(p, (p >> d1) + c1, (p >> d2) + c2)] == full[p], (tl, skew, nsym, p)
    assert checked > 20


def test_three_segments_fit_the_bench_tables():
    """The C5 keys / M frames of the bench's reads (zstd's own code lengths, HUF_buildCTable) fit the
    352 entries dec_huf_kernel keeps per frame -- with two segments they did not (410-480)."""
    import ctypes as C

    import _oracle as O

    M = O.model()
    M.z1m_huf_lengths.restype = C.c_uint
    M.z1m_huf_lengths.argtypes = [C.c_void_p, C.c_uint, C.c_void_p]
    for r in range(12):
        st = O.c5_streams(O.synth_read(r, 100000))
        for idx in (0, 2):  # keys, M
            h = np.bincount(np.frombuffer(st[idx], np.uint8), minlength=256).astype(np.uint32)
            nb = np.zeros(256, np.uint8)
            tl = int(M.z1m_huf_lengths(h.ctypes.data, int(np.nonzero(h)[0].max()), nb.ctypes.data))
            weights = [tl + 1 - int(v) if v else 0 for v in nb[: int(np.nonzero(h)[0].max()) + 1]]
            full, cnt, rank_start, before, order = _full_table(weights, tl)
            a = _compact_from_full(full, tl)
            assert a is not None and a[0][6] <= K_JOB_TAB_USE, (r, idx)
