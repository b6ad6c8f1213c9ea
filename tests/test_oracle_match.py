"""CPU: the matching oracle against the golden fixtures (descriptors from the
reference's in-tree VLFeat; expected matches from an independent numpy brute
force, see tests/golden/make_golden.py) and against numpy on edge cases."""
import json
import os

import numpy as np
import pytest

import _helpers as H
from golden.make_golden import numpy_match

abi = H.abi

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


def test_oracle_f32_integer_valued_equals_u8():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, size=(200, 128), dtype=np.uint8)
    b = rng.integers(0, 256, size=(150, 128), dtype=np.uint8)
    b[:20] = a[:20]
    for mode in (abi.SFM_MATCH_RATIO, abi.SFM_MATCH_MUTUAL):
        ui, ud = H.oracle_match_dense(a, b, mode)
        fi, fd = H.oracle_match_dense_f32(a.astype(np.float32), b.astype(np.float32), mode)
        np.testing.assert_array_equal(ui, fi)
        np.testing.assert_array_equal(np.where(ui >= 0, ud, -1).astype(np.float32), fd)


def test_oracle_f32_non_integer_against_float64():
    # away from near-ties the f32 restatement picks the float64 nearest neighbour
    rng = np.random.default_rng(4)
    a = rng.random((300, 128), dtype=np.float32) * 100
    b = rng.random((120, 128), dtype=np.float32) * 100
    fi, fd = H.oracle_match_dense_f32(a, b, abi.SFM_MATCH_MUTUAL)
    D = ((a[:, None, :].astype(np.float64) - b[None, :, :]) ** 2).sum(-1)
    nn = D.argmin(1)
    srt = np.sort(D, 1)
    clear = srt[:, 1] - srt[:, 0] > 1e-3 * srt[:, 0]
    mutual = D.argmin(0)[nn] == np.arange(len(a))
    want = np.where(mutual, nn, -1)
    np.testing.assert_array_equal(fi[clear], want[clear])
    ok = fi >= 0
    np.testing.assert_allclose(fd[ok], D[np.arange(len(a))[ok], fi[ok]], rtol=1e-5)
