"""The cell form's index decode (csrc/acm.hip ObsCells::get, r06) restated in
numpy binary64: i = trunc(c * RN(1 / ncx)), j = c - i ncx, one correction
when j >= ncx.  The claim: for every c < 2^32 and ncx < 2^32 this is
(c // ncx, c % ncx) -- the f64 quotient is within 2^-52 relative of c / ncx,
so its truncation can only fall one short, when c / ncx is an integer.
Checked on exact multiples (the only failing case of the bare truncation),
their neighbours and random cells, for grids up to the uint32 limit."""
import numpy as np


def decode(c, ncx):
    c = np.asarray(c, dtype=np.uint64)
    inv = np.float64(1.0) / np.float64(ncx)
    i = np.trunc(c.astype(np.float64) * inv).astype(np.uint64)
    j = c - i * np.uint64(ncx)
    fix = j >= np.uint64(ncx)
    i = np.where(fix, i + np.uint64(1), i)
    j = np.where(fix, j - np.uint64(ncx), j)
    return i, j


def test_decode_is_division():
    rng = np.random.default_rng(11)
    for ncx in [1, 2, 3, 7, 255, 256, 10_000, 10_001, 65_535, 99_991, 1 << 20, 4_000_000_007,
                *rng.integers(1, 1 << 24, 40).tolist()]:
        ncy = max(1, min((2 ** 32 - 1) // ncx, 1 << 16))
        total = ncx * ncy
        k = rng.integers(0, ncy, 20_000).astype(np.uint64)
        mult = k * np.uint64(ncx)
        cells = np.concatenate([mult, mult + 1, np.maximum(mult, 1) - 1,
                                rng.integers(0, total, 20_000).astype(np.uint64),
                                np.array([0, total - 1], dtype=np.uint64)])
        cells = cells[cells < total]
        i, j = decode(cells, ncx)
        assert np.array_equal(i, cells // np.uint64(ncx)), ncx
        assert np.array_equal(j, cells % np.uint64(ncx)), ncx


def test_bare_truncation_needs_the_correction():
    """Without the correction the decode is wrong somewhere (the bound is
    tight): exact multiples k ncx whose f64 quotient rounds below k."""
    wrong = 0
    for ncx in range(3, 3000):
        k = np.arange(1, 2000, dtype=np.uint64)
        c = k * np.uint64(ncx)
        i = np.trunc(c.astype(np.float64) * (1.0 / ncx)).astype(np.uint64)
        wrong += int((i != k).sum())
    assert wrong > 0
