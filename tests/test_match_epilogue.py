"""The exact matcher's top-2 update (csrc/match.hip, match_top2_kernel) keeps
the two smallest packed keys of a query with

    ta = med3(b1, x, y); b1 = min3(b1, x, y)
    tb = med3(b1, z, w); b1 = min3(b1, z, w)
    b2 = min3(b2, ta, tb)

over four keys at a time.  This checks the identity against a sorted
selection on the multiset (duplicates included: padding rows all carry
INT_MAX), so the GPU result equals Matcher_Regions' nearest / second-nearest
(sparseBuilder.cpp:919-921) whatever order the rows are visited in."""
import numpy as np


def _update4(b1, b2, x, y, z, w):
    ta = np.median(np.stack([b1, x, y]), axis=0).astype(np.int64)
    b1 = np.minimum(np.minimum(b1, x), y)
    tb = np.median(np.stack([b1, z, w]), axis=0).astype(np.int64)
    b1 = np.minimum(np.minimum(b1, z), w)
    b2 = np.minimum(np.minimum(b2, ta), tb)
    return b1, b2


def test_top2_update_matches_sorted_selection():
    rng = np.random.default_rng(0x70B2)
    for hi in (3, 8, 1 << 20):            # heavy ties, some ties, distinct
        keys = rng.integers(0, hi, size=(20000, 16), dtype=np.int64)
        keys[::7, 5:9] = np.iinfo(np.int32).max   # padding-row keys
        b1 = np.full(len(keys), np.iinfo(np.int32).max, np.int64)
        b2 = b1.copy()
        for j in range(0, 16, 4):
            b1, b2 = _update4(b1, b2, *(keys[:, j + t] for t in range(4)))
        s = np.sort(keys, axis=1)
        np.testing.assert_array_equal(b1, s[:, 0])
        np.testing.assert_array_equal(b2, s[:, 1])
