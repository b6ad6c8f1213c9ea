"""CPU: the matching oracle against the golden fixtures (descriptors from the
reference's in-tree VLFeat; expected matches from an independent numpy brute
force, see tests/golden/make_golden.py) and against numpy on edge cases."""
import json
import os

import numpy as np
import pytest

import _helpers as H
from golden.make_golden import numpy_match

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _views():
    return [np.fromfile(os.path.join(GOLD, f"vlfeat_view{k}.u8"), np.uint8).reshape(-1, 128)
            for k in range(3)]


def test_vlfeat_descriptor_statistics():
    # RootSIFT uchar from VLFeat: max ~125-130, ~11% zero bins (SURVEY §8c probe)
    for d in _views():
        assert d.shape[1] == 128 and len(d) > 200
        assert 100 <= d.max() <= 140
        assert 0.05 < (d == 0).mean() < 0.2


@pytest.mark.parametrize("mode", [0, 1])
def test_oracle_matches_golden(mode):
    views = _views()
    exp = json.load(open(os.path.join(GOLD, "vlfeat_matches.json")))
    assert exp["views"] == [len(v) for v in views]
    for i in range(3):
        for j in range(3):
            if i == j:
                continue
            e = exp["pairs"][f"{i}-{j}-{mode}"]
            oi, od = H.oracle_match_dense(views[i], views[j], mode)
            np.testing.assert_array_equal(oi, e["idx"])
            np.testing.assert_array_equal(od, e["d2"])
            if mode == 0:
                assert (oi >= 0).sum() > 50   # true correspondences exist


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("na,nb,hi", [(0, 3, 256), (3, 0, 256), (1, 5, 256), (2, 2, 256),
                                      (40, 70, 3), (300, 200, 256), (64, 64, 2)])
def test_oracle_vs_numpy_edge_cases(mode, na, nb, hi):
    rng = np.random.default_rng(na * 131 + nb + hi)
    a = rng.integers(0, hi, (na, 128), dtype=np.uint8)
    b = rng.integers(0, hi, (nb, 128), dtype=np.uint8)
    oi, od = H.oracle_match_dense(a, b, mode)
    ni, nd = numpy_match(a, b, mode)
    np.testing.assert_array_equal(oi, ni)
    np.testing.assert_array_equal(od, nd)


def test_ratio_uses_float32_square_of_0p8():
    # fl32(0.8f)^2 = 0.64000005 (not 0.64): d1 = 64, d2 = 100 is kept
    db = np.zeros((2, 128), np.uint8)
    db[0, :64] = 1
    db[1, :100] = 1
    q = np.zeros((1, 128), np.uint8)
    oi, od = H.oracle_match_dense(db, q, 0)
    assert oi[0] == 0 and od[0] == 64
