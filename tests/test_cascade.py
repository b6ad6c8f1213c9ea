"""Cascade-hashing matcher (SFM_MATCH_CASCADE): the reference's live default,
sparseBuilder.cpp:811-814,911-914 ("AUTO" -> Cascade_Hashing_Matcher_Regions).

Parity unpinned against OpenMVG itself (not vendored, not in the image); the
oracle (oracle/cascade_oracle.cpp) restates its published algorithm.  CPU
tests pin the oracle's projection matrix to an independent restatement of
libstdc++'s mt19937 / normal_distribution, and check the oracle's matches for
properties any cascade-hashing matcher has (self-matches, never better than
the exact NN, recall against the exact matcher).  GPU tests are bit-exact
against the oracle."""
import importlib
import math
import os

import numpy as np
import pytest

import _helpers as H

abi = H.abi
GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASC = abi.SFM_MATCH_CASCADE


# --- independent restatement of the projection RNG ---------------------------

def _mt19937(seed=5489):
    mt = [0] * 624
    mt[0] = seed
    for i in range(1, 624):
        mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
    idx = 624
    while True:
        if idx >= 624:
            for i in range(624):
                y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            idx = 0
        y = mt[idx]
        idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        yield y


def _normals(n):
    """libstdc++ normal_distribution<double>(0, 1) over mt19937: Marsaglia
    polar pairs (second value returned first, the first one cached), each
    uniform = generate_canonical<double, 53> = (x0 + x1 * 2^32) / 2^64."""
    g = _mt19937()

    def unif():
        x0 = next(g)
        x1 = next(g)
        r = (x0 + x1 * 4294967296.0) / 18446744073709551616.0
        return r if r < 1.0 else math.nextafter(1.0, 0.0)

    out, saved = [], None
    while len(out) < n:
        if saved is not None:
            out.append(saved)
            saved = None
            continue
        while True:
            x = 2.0 * unif() - 1.0
            y = 2.0 * unif() - 1.0
            r2 = x * x + y * y
            if r2 <= 1.0 and r2 != 0.0:
                break
        mult = math.sqrt(-2.0 * math.log(r2) / r2)
        saved = x * mult
        out.append(y * mult)
    return out


def test_projection_matrix_restated():
    import ctypes as C
    lib = H.oracle()
    p = np.zeros(188 * 128, np.float32)
    assert lib.orc_cascade_projections(p.ctypes.data_as(C.POINTER(C.c_float))) == 0
    ref = np.array(_normals(188 * 128), np.float64).astype(np.float32)
    np.testing.assert_array_equal(p, ref)
    assert abs(float(p.mean())) < 0.02 and 0.97 < float(p.std()) < 1.03


# --- oracle properties ---------------------------------------------------------

def _vlfeat():
    return [np.fromfile(os.path.join(GOLD, f"vlfeat_view{k}.u8"), np.uint8).reshape(-1, 128)
            for k in range(3)]


def test_oracle_self_matches():
    rng = np.random.default_rng(5)
    a = rng.integers(0, 130, (700, 128), dtype=np.uint8)
    idx, d = H.oracle_match_dense(a, a.copy(), CASC)
    m = idx >= 0
    assert m.mean() > 0.9
    np.testing.assert_array_equal(idx[m], np.nonzero(m)[0])
    assert (d[m] == 0).all()


def test_oracle_never_beats_exact_nn_and_recall():
    v = _vlfeat()
    for i, j in [(0, 1), (1, 2), (0, 2)]:
        ci, cd = H.oracle_match_dense(v[i], v[j], CASC)
        bi, bd = H.oracle_match_dense(v[i], v[j], abi.SFM_MATCH_RATIO)
        dI = v[i].astype(np.int32)
        for q in np.nonzero(ci >= 0)[0]:
            exact = ((dI - v[j][q].astype(np.int32)) ** 2).sum(1)
            assert cd[q] == exact[ci[q]]
            assert cd[q] >= exact.min()
        both = (bi >= 0) & (ci == bi)
        assert both.sum() >= 0.6 * (bi >= 0).sum(), (i, j, both.sum(), (bi >= 0).sum())


@pytest.mark.parametrize("na,nb", [(0, 4), (4, 0), (1, 3), (2, 2), (3, 1)])
def test_oracle_tiny_images_never_match(na, nb):
    # at most 2 database rows: "candidate_descriptors.size() <= NN" or < 2
    # distinct candidates -> no query is matched
    rng = np.random.default_rng(na + 10 * nb)
    a = rng.integers(0, 256, (na, 128), dtype=np.uint8)
    b = rng.integers(0, 256, (nb, 128), dtype=np.uint8)
    idx, d = H.oracle_match_dense(a, b, CASC)
    assert len(idx) == nb
    if na <= 2:
        assert (idx == -1).all() and (d == -1).all()


def test_oracle_pairs_equal_dense_on_two_images():
    v = _vlfeat()
    desc = np.concatenate([v[0], v[1]])
    off = np.array([0, len(v[0]), len(desc)], np.int64)
    c, i, j, d = H.oracle_match_pairs(desc, off, [[0, 1]], CASC)
    idx, dd = H.oracle_match_dense(v[0], v[1], CASC)
    q = np.nonzero(idx >= 0)[0]
    order = np.lexsort((q, idx[q]))
    np.testing.assert_array_equal(i, idx[q][order])
    np.testing.assert_array_equal(j, q[order])
    np.testing.assert_array_equal(d, dd[q][order])


# --- GPU parity -----------------------------------------------------------------

@pytest.fixture(scope="module")
def ctx():
    api = importlib.import_module("3dreconstruction_amd.api")
    c = api.Context(0)
    yield c
    c.close()


def _api():
    return importlib.import_module("3dreconstruction_amd.api")


@pytest.mark.gpu
def test_gpu_dense_vlfeat(ctx):
    v = _vlfeat()
    for i in range(3):
        for j in range(3):
            if i == j:
                continue
            gi, gd = _api().match_dense(ctx, v[i], v[j], CASC)
            oi, od = H.oracle_match_dense(v[i], v[j], CASC)
            np.testing.assert_array_equal(gi, oi)
            np.testing.assert_array_equal(gd, od)
            assert (gi >= 0).sum() > 30


@pytest.mark.gpu
@pytest.mark.parametrize("na,nb,hi", [(0, 5, 256), (5, 0, 256), (1, 7, 256), (2, 2, 256),
                                      (3, 3, 256), (37, 300, 256), (513, 1000, 130),
                                      (600, 600, 3), (300, 300, 1),
                                      # > kCascLdsMaxN rows: the global-table kernel
                                      (6000, 700, 130)])
def test_gpu_dense_random(ctx, na, nb, hi):
    rng = np.random.default_rng(na * 7919 + nb + hi)
    a = rng.integers(0, hi, (na, 128), dtype=np.uint8)
    b = rng.integers(0, hi, (nb, 128), dtype=np.uint8)
    if hi == 130:
        m = min(na, nb) // 2
        b[:m] = a[:m]
    gi, gd = _api().match_dense(ctx, a, b, CASC)
    oi, od = H.oracle_match_dense(a, b, CASC)
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gd, od)


@pytest.mark.gpu
def test_gpu_plan_vs_oracle_ragged_and_rehash(ctx):
    sizes = [700, 0, 1, 3, 257, 1200, 512, 64, 900, 2]
    d = H.synth_descriptors(len(sizes), 1200)
    rows, off = [], [0]
    for k, n in enumerate(sizes):
        rows.append(d[k * 1200:k * 1200 + n])
        off.append(off[-1] + n)
    desc = np.concatenate(rows)
    off = np.array(off, np.int64)
    full = np.array([(i, j) for i in range(len(sizes)) for j in range(i + 1, len(sizes))], np.int32)
    sub = full[(full[:, 0] >= 4) & (full[:, 1] <= 8)]   # other images -> other zero-mean
    plan = _api().MatchPlan(ctx, desc, off)
    try:
        for pairs in (full, sub, full):
            tot = plan.run(pairs, mode=CASC)
            c, i, j, dd = plan.fetch()
            oc, oi, oj, od = H.oracle_match_pairs(desc, off, pairs, CASC)
            assert tot == int(oc.sum()) and tot > 100
            np.testing.assert_array_equal(c, oc)
            np.testing.assert_array_equal(i, oi)
            np.testing.assert_array_equal(j, oj)
            np.testing.assert_array_equal(dd, od)
        # a list split into parts (ranks / batches) after cascade_index(full)
        # matches exactly as the whole list
        plan.cascade_index(full)
        oc, oi, oj, od = H.oracle_match_pairs(desc, off, full, CASC)
        got = [[], [], [], []]
        for part in (full[:7], full[7:30], full[30:]):
            plan.run(part, mode=CASC)
            for k, v in enumerate(plan.fetch()):
                got[k].append(v)
        for k, v in enumerate((oc, oi, oj, od)):
            np.testing.assert_array_equal(np.concatenate(got[k]), v)
    finally:
        plan.close()
