"""Host restatement of the lane-parallel FSE compression table build (pgn_zenc.h fse_build_ctable_small,
the weight alphabet of HUF_writeCTable) against the serial FSE_buildCTable_wksp of libzstd 1.4.x.

Serial: low-probability (-1) symbols take the top positions in symbol order, the others are spread
along positions (j * step) & mask skipping those above highThreshold, and the state table numbers
each symbol's positions in increasing order.  Parallel: visit j's slot is its rank among the valid
visits, its symbol the count of symbols whose cumulative normal count is <= that slot, and an entry's
state the symbol's cumul plus its rank among the symbol's entries.  Random normalized counts (table
logs 5 and 6, up to 13 symbols, with -1 and 0 entries) must give identical tables and deltas.
"""
import numpy as np


def _serial(norm, table_log):
    ts = 1 << table_log
    mask = ts - 1
    step = (ts >> 1) + (ts >> 3) + 3
    ht = ts - 1
    sym_tab = [None] * ts
    cumul = [0] * (len(norm) + 1)
    for u in range(1, len(norm) + 1):
        if norm[u - 1] == -1:
            cumul[u] = cumul[u - 1] + 1
            sym_tab[ht] = u - 1
            ht -= 1
        else:
            cumul[u] = cumul[u - 1] + norm[u - 1]
    pos = 0
    for s, f in enumerate(norm):
        for _ in range(max(f, 0)):
            sym_tab[pos] = s
            pos = (pos + step) & mask
            while pos > ht:
                pos = (pos + step) & mask
    assert pos == 0
    state = [None] * ts
    c = list(cumul)
    for u in range(ts):
        s = sym_tab[u]
        state[c[s]] = ts + u
        c[s] += 1
    return sym_tab, state, cumul[:len(norm)]


def _parallel(norm, table_log):
    ts = 1 << table_log
    mask = ts - 1
    step = (ts >> 1) + (ts >> 3) + 3
    n = len(norm)
    low = [v == -1 for v in norm]
    cnt = [1 if low[s] else max(norm[s], 0) for s in range(n)]
    excl = [sum(cnt[:s]) for s in range(n)]
    sym_tab = [None] * ts
    for s in range(n):
        if low[s]:
            sym_tab[ts - 1 - sum(low[:s])] = s
    ht = ts - 1 - sum(low)
    nincl = [sum(0 if low[q] else cnt[q] for q in range(s + 1)) for s in range(n)]
    valid = [((j * step) & mask) <= ht for j in range(ts)]
    for j in range(ts):
        if valid[j]:
            k = sum(valid[:j])
            sym_tab[(j * step) & mask] = sum(1 for q in range(n) if nincl[q] <= k)
    state = [None] * ts
    for u in range(ts):
        s = sym_tab[u]
        rank = sum(1 for v in range(u) if sym_tab[v] == s)
        state[excl[s] + rank] = ts + u
    return sym_tab, state, excl


def _random_norm(rng, table_log):
    ts = 1 << table_log
    while True:
        n = int(rng.integers(2, 14))
        norm = [0] * n
        left = ts
        for s in rng.permutation(n)[: int(rng.integers(2, n + 1))]:
            norm[s] = -1 if rng.random() < 0.25 else 1
        left -= sum(1 for v in norm if v != 0)
        nz = [s for s in range(n) if norm[s] > 0]
        if not nz or left < 0:
            continue
        while left > 0:
            s = nz[int(rng.integers(0, len(nz)))]
            add = int(rng.integers(1, left + 1))
            norm[s] += add
            left -= add
        return norm


def test_parallel_fse_table_equals_serial():
    rng = np.random.default_rng(17)
    for table_log in (5, 6):
        for _ in range(300):
            norm = _random_norm(rng, table_log)
            assert _serial(norm, table_log) == _parallel(norm, table_log), norm
