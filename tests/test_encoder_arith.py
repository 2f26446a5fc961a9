"""Host checks of the integer shortcuts the encoder kernels take (no GPU).

The literal histogram (pgn_zenc.h compress_literals_wave) finds a 16-byte block's Huffman segment
as __umulhi(i, ceil(2^32 / segSize)) instead of i / segSize.  That is exact for every block offset a
literals section has: i < 2^17 (a block is at most 128 KiB, ZSTD_BLOCKSIZE_MAX) and 64 <= segSize <=
2^15 (segSize = ceil(n / 4) for n >= 256, or n itself for 64 <= n < 256).
"""
import numpy as np


def _magic(d: int) -> int:
    return 0xFFFFFFFF // d + 1


def test_segment_multiply_high_is_exact():
    rng = np.random.default_rng(5)
    d = np.arange(64, 32769, dtype=np.uint64)
    m = np.array([_magic(int(x)) for x in d], dtype=np.uint64)
    n = np.minimum(4 * d, 131072)
    # the largest offsets (where the reciprocal's error is largest), a spread of small ones, random
    k = 16 * np.arange(1, 65, dtype=np.uint64)[None, :]
    top = np.where(k <= n[:, None], n[:, None] - np.minimum(k, n[:, None]), 0).astype(np.uint64)
    rnd = (rng.integers(0, 1 << 30, size=(d.size, 64)).astype(np.uint64) % n[:, None]) & ~np.uint64(15)
    low = np.broadcast_to(16 * np.arange(64, dtype=np.uint64)[None, :], (d.size, 64))
    for i in (top, rnd, low):
        q = (i * m[:, None]) >> np.uint64(32)
        assert np.array_equal(q, i // d[:, None])


def test_segment_multiply_high_boundaries():
    # every segment boundary k * segSize and the block just below it, for the bench's stream sizes
    for n in (256, 1114, 16570, 25000, 63605, 100000, 131072):
        d = (n + 3) // 4
        m = _magic(d)
        for k in range(1, 4):
            for i in (k * d - 1, k * d, k * d + 1):
                if 0 <= i < n:
                    assert (i * m) >> 32 == i // d
