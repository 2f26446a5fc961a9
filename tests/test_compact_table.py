"""Host restatement of the deferred Huffman job's compact table (pgn_hufjob.h), checked two ways.

huf_defer_body builds it from the full single-symbol decode table (HUF_readDTableX1: weight w owns the
entries [rankStart[w], rankStart[w] + cnt[w] << (w - 1)), symbols in (weight, symbol) order): it counts
the entries whose code is longer than K = tl - d for d = 1..4, keeps the smallest table, and gathers
entry j from full[j < T ? j : (j - Cc) << d].  dec_frame_fast (pgn_zdec.h huf_build_dtable_body with a
job table) computes the same entries from the ranks alone: T_d = rankStart[d + 1], and entry idx belongs
to the last weight whose range starts at or below it.  Both are restated here over random weight sets
(every table log 5..11, skewed and flat) and must agree entry for entry, with the same K and Cc.
"""
import numpy as np

K_JOB_TAB_USE = 504


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


def _compact_from_full(full, tl):
    tsz = 1 << tl
    ts = [sum(1 for e in full if e[1] + d > tl) for d in range(1, 5)]
    K, T, size = tl, 0, tsz
    for d in range(1, 5):
        if d >= tl:
            break
        t = ts[d - 1]
        sz = t + ((tsz - t) >> d)
        if sz < size:
            size, K, T = sz, tl - d, t
    if size > K_JOB_TAB_USE:
        return None
    d = tl - K
    Cc = T - (T >> d)
    return K, Cc, [full[j if j < T else (j - Cc) << d] for j in range(size)]


def _compact_from_ranks(cnt, rank_start, before, order, tl):
    tsz = 1 << tl
    K, T, size = tl, 0, tsz
    for d in range(1, 5):
        if d >= tl:
            break
        t = rank_start[d + 1]
        sz = t + ((tsz - t) >> d)
        if sz < size:
            size, K, T = sz, tl - d, t
    if size > K_JOB_TAB_USE:
        return None
    d = tl - K
    Cc = T - (T >> d)
    out = []
    for j in range(size):
        idx = j if j < T else (j - Cc) << d
        w = rs0 = bf = 0
        for ww in range(1, 13):
            if ww <= tl and cnt[ww] and rank_start[ww] <= idx:
                w, rs0, bf = ww, rank_start[ww], before[ww]
        out.append((order[bf + ((idx - rs0) >> (w - 1))][1], tl + 1 - w))
    return K, Cc, out


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
                checked += a is not None
    assert checked > 20
