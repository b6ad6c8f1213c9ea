"""GPU parity tests for the HIP matcher against the CPU oracle (bit-exact
integer indices and squared distances)."""
import importlib

import numpy as np
import pytest

import _helpers as H

pytestmark = pytest.mark.gpu
abi = H.abi
api = importlib.import_module("3dreconstruction_amd.api")


@pytest.fixture(scope="module")
def ctx():
    c = api.Context(0)
    yield c
    c.close()


def _rand(rng, n, hi=256):
    return rng.integers(0, hi, size=(n, 128), dtype=np.uint8)


@pytest.mark.parametrize("mode", [abi.SFM_MATCH_RATIO, abi.SFM_MATCH_MUTUAL])
@pytest.mark.parametrize("na,nb", [(0, 5), (5, 0), (1, 7), (2, 2), (37, 300), (256, 256),
                                   (300, 37), (513, 1000), (1024, 2048)])
def test_dense_random(ctx, mode, na, nb):
    rng = np.random.default_rng(na * 7919 + nb)
    a, b = _rand(rng, na), _rand(rng, nb)
    gi, gd = api.match_dense(ctx, a, b, mode)
    oi, od = H.oracle_match_dense(a, b, mode)
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gd, od)


@pytest.mark.parametrize("mode", [abi.SFM_MATCH_RATIO, abi.SFM_MATCH_MUTUAL])
def test_dense_synthetic_sift(ctx, mode):
    d = H.synth_descriptors(2, 4096)
    a, b = d[:4096], d[4096:]
    gi, gd = api.match_dense(ctx, a, b, mode)
    oi, od = H.oracle_match_dense(a, b, mode)
    assert (oi >= 0).sum() > 100
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gd, od)


@pytest.mark.parametrize("mode", [abi.SFM_MATCH_RATIO, abi.SFM_MATCH_MUTUAL])
def test_ties_and_extremes(ctx, mode):
    rng = np.random.default_rng(5)
    base = _rand(rng, 64, hi=4)                    # many exact ties
    a = np.concatenate([base, base, np.zeros((3, 128), np.uint8), np.full((3, 128), 255, np.uint8)])
    b = np.concatenate([base[::-1], np.full((2, 128), 255, np.uint8), np.zeros((2, 128), np.uint8)])
    gi, gd = api.match_dense(ctx, a, b, mode)
    oi, od = H.oracle_match_dense(a, b, mode)
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gd, od)


def test_ratio_threshold_boundary(ctx):
    # d1 = 64, d2 = 100: kept only because the threshold is fl32(0.8f)^2 =
    # 0.64000005 (64 < 64.000005); with an exact 0.64 it would be dropped.
    q = np.zeros((1, 128), np.uint8)
    db = np.zeros((2, 128), np.uint8)
    db[0, :64] = 1
    db[1, :100] = 1
    gi, gd = api.match_dense(ctx, db, q, abi.SFM_MATCH_RATIO)
    assert gi[0] == 0 and gd[0] == 64
    db[0, :65] = 1          # d1 = 65 -> dropped
    gi, gd = api.match_dense(ctx, db, q, abi.SFM_MATCH_RATIO)
    assert gi[0] == -1


@pytest.mark.parametrize("mode", [abi.SFM_MATCH_RATIO, abi.SFM_MATCH_MUTUAL])
def test_all_pairs_plan(ctx, mode):
    sizes = [700, 0, 257, 1024, 1, 513]
    rng = np.random.default_rng(11)
    syn = H.synth_descriptors(6, 1024)
    desc = np.concatenate([syn[k * 1024:k * 1024 + n] for k, n in enumerate(sizes)])
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    pairs = api.exhaustive_pairs(len(sizes))
    pairs = np.concatenate([pairs, pairs[::-1, ::-1]])  # both orientations
    plan = api.MatchPlan(ctx, desc, off)
    total = plan.run(pairs, mode)
    counts, i, j, d = plan.fetch()
    lib = H.oracle()
    oc = np.zeros(len(pairs), np.int64)
    lib.orc_match_pairs(abi.ptr(desc, abi.u8p), abi.ptr(off, abi.i64p), len(sizes),
                        abi.ptr(pairs, abi.i32p), len(pairs), mode, 0.8, 4,
                        abi.ptr(oc, abi.i64p), None, None, None)
    n = int(oc.sum())
    oi = np.zeros(n, np.uint32); oj = np.zeros(n, np.uint32); od = np.zeros(n, np.int32)
    lib.orc_match_pairs(abi.ptr(desc, abi.u8p), abi.ptr(off, abi.i64p), len(sizes),
                        abi.ptr(pairs, abi.i32p), len(pairs), mode, 0.8, 4,
                        abi.ptr(oc, abi.i64p), abi.ptr(oi, abi.u32p), abi.ptr(oj, abi.u32p),
                        abi.ptr(od, abi.i32p))
    np.testing.assert_array_equal(counts, oc)
    np.testing.assert_array_equal(i, oi)
    np.testing.assert_array_equal(j, oj)
    np.testing.assert_array_equal(d, od)
    assert total == n
    assert plan.digest() == api.match_digest(oc, oi, oj, od)
    plan.close()


# ---- float descriptors (cv::Mat CV_32F behind LocalFrame/GlobalFrame) ------

def _rootsift_f32(rng, n):
    """Non-integer float descriptors (L1-normalised, square-rooted, x512)."""
    v = rng.gamma(0.6, 1.0, size=(n, 128)).astype(np.float64)
    v /= v.sum(1, keepdims=True) + 1e-12
    return (512.0 * np.sqrt(v)).astype(np.float32)


@pytest.mark.parametrize("mode", [abi.SFM_MATCH_RATIO, abi.SFM_MATCH_MUTUAL])
def test_dense_f32_integer_valued_is_the_u8_path(ctx, mode):
    # cv::SIFT stores saturate_cast<uchar> values in its float rows: converted
    # exactly, same indices as the u8 matcher, distances exact integers
    d = H.synth_descriptors(2, 1500)
    a, b = d[:1500], d[1500:][:1100]
    gi, gd = api.match_dense_f32(ctx, a.astype(np.float32), b.astype(np.float32), mode)
    ui, ud = api.match_dense(ctx, a, b, mode)
    oi, od = H.oracle_match_dense_f32(a.astype(np.float32), b.astype(np.float32), mode)
    np.testing.assert_array_equal(gi, ui)
    np.testing.assert_array_equal(gd, np.where(ui >= 0, ud, -1).astype(np.float32))
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))


@pytest.mark.parametrize("mode", [abi.SFM_MATCH_RATIO, abi.SFM_MATCH_MUTUAL])
@pytest.mark.parametrize("na,nb", [(0, 5), (5, 0), (1, 7), (2, 2), (300, 37), (777, 1029)])
def test_dense_f32_non_integer_bit_exact(ctx, mode, na, nb):
    rng = np.random.default_rng(na * 31 + nb)
    a, b = _rootsift_f32(rng, na), _rootsift_f32(rng, nb)
    if na > 4 and nb > 4:
        b[:4] = a[:4] + np.float32(0.25)       # near-duplicates: real matches
        a[na // 2] = a[0]                      # an exact tie for query 0 in RATIO
    gi, gd = api.match_dense_f32(ctx, a, b, mode)
    oi, od = H.oracle_match_dense_f32(a, b, mode)
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gd.view(np.uint32), od.view(np.uint32))


def test_plan_f32_collection(ctx):
    rng = np.random.default_rng(77)
    sizes = [300, 0, 129, 513, 1]
    desc = _rootsift_f32(rng, sum(sizes))
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    pairs = api.exhaustive_pairs(len(sizes))
    plan = api.MatchPlan(ctx, desc, off)
    for mode in (abi.SFM_MATCH_RATIO, abi.SFM_MATCH_MUTUAL):
        plan.run(pairs, mode)
        counts, i, j, d = plan.fetch()
        assert d.dtype == np.float32
        k = 0
        for p, (I, J) in enumerate(pairs):
            dI, dJ = desc[off[I]:off[I + 1]], desc[off[J]:off[J + 1]]
            oi, od = H.oracle_match_dense_f32(dI, dJ, mode)
            q = np.nonzero(oi >= 0)[0]
            if mode == abi.SFM_MATCH_RATIO:
                want = sorted(zip(oi[q].tolist(), q.tolist(), od[q].view(np.uint32).tolist()))
            else:
                want = sorted(zip(q.tolist(), oi[q].tolist(), od[q].view(np.uint32).tolist()))
            got = list(zip(i[k:k + counts[p]].tolist(), j[k:k + counts[p]].tolist(),
                           d[k:k + counts[p]].view(np.uint32).tolist()))
            assert got == want, (p, I, J)
            k += counts[p]
    with pytest.raises(RuntimeError):
        plan.run(pairs, abi.SFM_MATCH_CASCADE)     # hashing needs integer descriptors
    plan.close()
