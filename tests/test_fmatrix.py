"""Geometric filter: GeometricFilter_FMatrix_AC(4.0,
2048) of sparseBuilder::filter() (src/sparseBuilder/sparseBuilder.cpp:1179-1186)
= OpenMVG ACRANSAC over the 7-point fundamental-matrix kernel.

OpenMVG is un-vendored, so the oracle (oracle/fmat_oracle.cpp) restates its
published code: PARITY UNPINNED against OpenMVG itself.  Pinned here on the
CPU: the sampler's random stream (std::mt19937 + libstdc++
uniform_int_distribution, which the GPU restates as Lemire's method) against
an independent numpy restatement, the exact-operation log10 / cube root
against libm, the 7-point solver's algebra, and the filter's behaviour on
scenes with a known epipolar geometry.  On the GPU: sfm_fmatrix_ac equals the
oracle bit for bit (inlier index lists in residual order, F, thresholds,
NFA, iteration counts).
"""
import ctypes as C
import math

import numpy as np
import pytest

import _helpers as H
from _helpers import abi, api


def _orc():
    lib = H.oracle()
    if not getattr(lib, "_fmat_sig", False):
        lib.orc_fmatrix_ac.restype = C.c_int
        lib.orc_fmatrix_ac.argtypes = [C.c_int64, abi.i64p, abi.f64p, abi.i32p, C.POINTER(abi.FMatrixOpts),
                                       C.POINTER(abi.FMatrixResult), abi.i32p, C.c_int32]
        lib.orc_uniform_draws.restype = C.c_int
        lib.orc_uniform_draws.argtypes = [abi.u32p, abi.u32p, C.c_int64, abi.u32p]
        lib.orc_det_math.restype = C.c_int
        lib.orc_det_math.argtypes = [C.c_int32, abi.f64p, C.c_int64, abi.f64p]
        lib.orc_seven_point.restype = C.c_int
        lib.orc_seven_point.argtypes = [abi.f64p, abi.f64p, abi.f64p, abi.i32p]
        lib._fmat_sig = True
    return lib


def oracle_fmatrix_ac(xy_list, wh, opts=None, threads=8):
    lib = _orc()
    off, xy, wh = api._fmatrix_inputs(xy_list, wh)
    n_pairs = len(off) - 1
    res = (abi.FMatrixResult * max(n_pairs, 1))()
    inl = np.full(max(int(off[-1]), 1), -1, np.int32)
    assert lib.orc_fmatrix_ac(n_pairs, abi.ptr(off, abi.i64p), abi.ptr(xy, abi.f64p), abi.ptr(wh, abi.i32p),
                              C.byref(opts or api.fmatrix_opts()), res, abi.ptr(inl, abi.i32p), threads) == 0
    return api._fmatrix_outputs(off, res, inl)


def _rot(w):
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


def synth_pair(n, outlier_frac, seed, w=1920, h=1080, f=1400.0, noise=0.5, baseline=0.6):
    """Two views of random points: (n, 4) pixel correspondences, the true F
    (x_J' F x_I = 0) and the inlier mask."""
    rng = np.random.default_rng(seed)
    K = np.array([[f, 0, w / 2], [0, f, h / 2], [0, 0, 1.0]])
    R2 = _rot(rng.normal(0, 0.15, 3))
    t2 = np.array([-baseline, rng.normal(0, 0.1), rng.normal(0, 0.1)])
    X = np.stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(5, 12, n)], 1)
    p1 = (K @ X.T).T
    p2 = (K @ (R2 @ X.T + t2[:, None])).T
    u1 = p1[:, :2] / p1[:, 2:] + rng.normal(0, noise, (n, 2))
    u2 = p2[:, :2] / p2[:, 2:] + rng.normal(0, noise, (n, 2))
    out = rng.random(n) < outlier_frac
    u2[out] = np.stack([rng.uniform(0, w, out.sum()), rng.uniform(0, h, out.sum())], 1)
    tx = np.array([[0, -t2[2], t2[1]], [t2[2], 0, -t2[0]], [-t2[1], t2[0], 0]])
    Kinv = np.linalg.inv(K)
    F = Kinv.T @ tx @ R2 @ Kinv
    return np.concatenate([u1, u2], 1), F / np.linalg.norm(F), ~out


def epi_dist(F, xy):
    x1 = np.concatenate([xy[:, :2], np.ones((len(xy), 1))], 1)
    x2 = np.concatenate([xy[:, 2:], np.ones((len(xy), 1))], 1)
    l = x1 @ F.T
    return np.abs(np.sum(x2 * l, 1)) / np.hypot(l[:, 0], l[:, 1])


# ---------------------------------------------------------------- CPU ------


def _mt19937_raw(n):
    """std::mt19937(5489) outputs: numpy's MT19937 with init_genrand seeding"""
    bg = np.random.MT19937()
    bg._legacy_seeding(5489)
    return bg.random_raw(n).astype(np.uint64)


def _lemire(stream, lo, hi):
    """libstdc++ uniform_int_distribution<uint32_t> on 32-bit outputs (the GPU's restatement)"""
    out, pos = [], 0
    for a, b in zip(lo, hi):
        rng_ = (int(b) - int(a)) & 0xFFFFFFFF
        if rng_ == 0xFFFFFFFF:
            out.append((a + int(stream[pos])) & 0xFFFFFFFF)
            pos += 1
            continue
        r = rng_ + 1
        prod = int(stream[pos]) * r
        pos += 1
        low = prod & 0xFFFFFFFF
        if low < r:
            thr = ((1 << 32) - r) % r
            while low < thr:
                prod = int(stream[pos]) * r
                pos += 1
                low = prod & 0xFFFFFFFF
        out.append(int(a) + (prod >> 32))
    return np.array(out, np.uint32)


def test_sampler_stream_is_libstdcxx():
    rng = np.random.default_rng(3)
    n = 4000
    lo = rng.integers(0, 8, n).astype(np.uint32)
    span = rng.choice([1, 7, 20, 1000, 3_000_000_000, 0xFFFFFFFF - 8], n)
    hi = np.minimum(lo.astype(np.uint64) + span.astype(np.uint64), 0xFFFFFFFF).astype(np.uint32)
    got = np.zeros(n, np.uint32)
    assert _orc().orc_uniform_draws(abi.ptr(lo, abi.u32p), abi.ptr(hi, abi.u32p), n, abi.ptr(got, abi.u32p)) == 0
    want = _lemire(_mt19937_raw(3 * n), lo, hi)
    assert np.array_equal(got, want)


def test_exact_operation_math():
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(1e-8, 1e8, 2000), np.arange(1, 3000, dtype=np.float64),
                        [1.1920928955078125e-07, 1e-300, 1e300]])
    out = np.zeros_like(x)
    assert _orc().orc_det_math(0, abi.ptr(x, abi.f64p), len(x), abi.ptr(out, abi.f64p)) == 0
    assert np.max(np.abs(out - np.log10(x)) / np.maximum(1.0, np.abs(np.log10(x)))) < 4e-16
    assert _orc().orc_det_math(1, abi.ptr(x, abi.f64p), len(x), abi.ptr(out, abi.f64p)) == 0
    assert np.max(np.abs(out - np.cbrt(x)) / np.cbrt(x)) < 4e-16


def test_seven_point_models_fit_the_sample():
    lib = _orc()
    for seed in range(20):
        xy, F, _ = synth_pair(7, 0.0, seed, noise=0.0)
        # normalised as the filter normalises (1/sqrt(w h), centred)
        s = 1 / math.sqrt(1920 * 1080)
        x1 = np.ascontiguousarray((xy[:, :2] - [960, 540]) * s)
        x2 = np.ascontiguousarray((xy[:, 2:] - [960, 540]) * s)
        Fs = np.zeros(27)
        nm = C.c_int32()
        assert lib.orc_seven_point(abi.ptr(x1, abi.f64p), abi.ptr(x2, abi.f64p), abi.ptr(Fs, abi.f64p),
                                   C.byref(nm)) == 0
        assert nm.value in (1, 3)
        h1 = np.concatenate([x1, np.ones((7, 1))], 1)
        h2 = np.concatenate([x2, np.ones((7, 1))], 1)
        T = np.array([[s, 0, -960 * s], [0, s, -540 * s], [0, 0, 1]])
        Ftrue = np.linalg.inv(T).T @ F @ np.linalg.inv(T)
        Ftrue /= np.linalg.norm(Ftrue)
        best = 9.0
        for k in range(nm.value):
            M = Fs[9 * k:9 * k + 9].reshape(3, 3)
            M = M / np.linalg.norm(M)
            assert np.max(np.abs(np.sum(h2 * (h1 @ M.T), 1))) < 1e-9
            assert abs(np.linalg.det(M)) < 1e-9
            best = min(best, np.linalg.norm(M - Ftrue), np.linalg.norm(M + Ftrue))
        assert best < 1e-6   # one of the roots is the true geometry (noise-free)


@pytest.mark.parametrize("outliers", [0.0, 0.3, 0.6])
def test_oracle_recovers_epipolar_geometry(outliers):
    xy, F, good = synth_pair(600, outliers, 11)
    r = oracle_fmatrix_ac([xy], [(1920, 1080, 1920, 1080)])[0]
    assert r["n_inliers"] > 17 and r["min_nfa"] < 0
    inl = np.zeros(len(xy), bool)
    inl[r["inliers"]] = True
    assert len(set(r["inliers"].tolist())) == r["n_inliers"]
    tp = (inl & good).sum()
    assert tp / good.sum() > 0.9                        # recall of true correspondences
    assert (inl & ~good).sum() <= 0.02 * len(xy) + 2    # few outliers survive
    assert r["error_max"] <= 4.0 + 1e-9                  # the a-contrario bound
    d = epi_dist(r["F"], xy[r["inliers"]])
    assert np.all(d <= r["error_max"] * (1 + 1e-6) + 1e-9)
    # inliers in OpenMVG's order: ascending residual
    assert np.all(np.diff(d) >= -1e-6 * (1 + d[1:]))


def test_oracle_edge_cases():
    rng = np.random.default_rng(2)
    noise = np.stack([rng.uniform(0, 1920, 300), rng.uniform(0, 1080, 300),
                      rng.uniform(0, 1920, 300), rng.uniform(0, 1080, 300)], 1)
    same = np.tile([[100.0, 200.0, 300.0, 400.0]], (40, 1))
    res = oracle_fmatrix_ac([np.zeros((0, 4)), np.ones((5, 4)), np.ones((7, 4)), noise, same],
                            [(1920, 1080, 1920, 1080)] * 5)
    for r in res[:3]:
        assert r["n_inliers"] == 0 and r["iterations"] == 0
    assert res[3]["n_inliers"] == 0 or res[3]["n_inliers"] < 60   # pure clutter: nothing meaningful
    assert res[4]["n_inliers"] == 0                                   # one repeated point: degenerate
    a = oracle_fmatrix_ac([noise], [(1920, 1080, 1920, 1080)], threads=1)[0]
    b = oracle_fmatrix_ac([noise], [(1920, 1080, 1920, 1080)], threads=4)[0]
    assert a["iterations"] == b["iterations"] and np.array_equal(a["inliers"], b["inliers"])


# ---------------------------------------------------------------- GPU ------


def _batch(sizes_fracs, seed0=100):
    xs, whs = [], []
    for k, (n, frac) in enumerate(sizes_fracs):
        w, h = (1920, 1080) if k % 2 == 0 else (1280, 960)
        xy, _, _ = synth_pair(n, frac, seed0 + k, w=w, h=h) if n else (np.zeros((0, 4)), None, None)
        xs.append(xy)
        whs.append((w, h, w, h))
    return xs, whs


def _same(g, o):
    assert g["iterations"] == o["iterations"]
    assert g["n_inliers"] == o["n_inliers"]
    assert np.array_equal(g["inliers"], o["inliers"])
    assert np.array_equal(g["F"].view(np.uint64), o["F"].view(np.uint64))
    assert g["error_max"] == o["error_max"] or (math.isinf(g["error_max"]) and math.isinf(o["error_max"]))
    assert g["min_nfa"] == o["min_nfa"] or (math.isinf(g["min_nfa"]) and math.isinf(o["min_nfa"]))


@pytest.fixture(scope="module")
def ctx():
    c = api.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
def test_gpu_fmatrix_bit_exact(ctx):
    xs, whs = _batch([(0, 0), (5, 0), (8, 0.0), (20, 0.1), (60, 0.5), (300, 0.3), (1000, 0.2),
                      (2500, 0.4), (4000, 0.1), (150, 0.9), (800, 0.0)])
    got = api.fmatrix_ac(ctx, xs, whs)
    want = oracle_fmatrix_ac(xs, whs)
    for g, o in zip(got, want):
        _same(g, o)
    assert sum(g["n_inliers"] > 0 for g in got) >= 7


@pytest.mark.gpu
def test_gpu_fmatrix_degenerate_and_clutter(ctx):
    rng = np.random.default_rng(9)
    clutter = np.stack([rng.uniform(0, 1920, 400), rng.uniform(0, 1080, 400),
                        rng.uniform(0, 1920, 400), rng.uniform(0, 1080, 400)], 1)
    same = np.tile([[100.0, 200.0, 300.0, 400.0]], (40, 1))
    line = np.stack([np.linspace(0, 1900, 50), np.full(50, 500.0), np.linspace(10, 1910, 50), np.full(50, 520.0)], 1)
    xs = [clutter, same, line]
    whs = [(1920, 1080, 1920, 1080)] * 3
    for g, o in zip(api.fmatrix_ac(ctx, xs, whs), oracle_fmatrix_ac(xs, whs)):
        _same(g, o)


@pytest.mark.gpu
def test_gpu_fmatrix_options_and_global_sort(ctx):
    # fewer iterations, a tighter bound; one pair above the LDS sort capacity
    xs, whs = _batch([(9000, 0.2), (500, 0.3)], seed0=300)
    o = api.fmatrix_opts(precision=2.0, max_iterations=300)
    for g, w in zip(api.fmatrix_ac(ctx, xs, whs, o), oracle_fmatrix_ac(xs, whs, o)):
        _same(g, w)


@pytest.mark.gpu
def test_gpu_fmatrix_mixed_global_and_lds_sort(ctx):
    # two pairs above the LDS sort capacity (different global buffer sizes,
    # packed by prefix sum) between small pairs that keep the LDS sort
    xs, whs = _batch([(300, 0.3), (17000, 0.2), (40, 0.1), (9000, 0.3), (700, 0.5), (0, 0), (2000, 0.2)],
                     seed0=700)
    o = api.fmatrix_opts(precision=4.0, max_iterations=200)
    for g, w in zip(api.fmatrix_ac(ctx, xs, whs, o), oracle_fmatrix_ac(xs, whs, o)):
        _same(g, w)


def _stage(d, n_views=4, n_pts=400, seed=21):
    """sfm_data.json + <stem>.feat of n_views 640x480 views of one scene and a
    matches.putative.bin of every pair: true correspondences plus 25 % wrong
    matches, in (i, j) order."""
    from test_mvg_io import write_feat, write_sfm_data
    rng = np.random.default_rng(seed)
    w, h, f = 640, 480, 500.0
    K = np.array([[f, 0, w / 2], [0, f, h / 2], [0, 0, 1.0]])
    X = np.stack([rng.uniform(-2, 2, n_pts), rng.uniform(-1.5, 1.5, n_pts), rng.uniform(6, 10, n_pts)], 1)
    names = [f"v{k}.jpg" for k in range(n_views)]
    write_sfm_data(d / "sfm_data.json", names)
    perms, kps = [], []
    for v in range(n_views):
        R = _rot(np.array([0.0, -0.05 * v, 0.01 * v]))
        t = np.array([-0.4 * v, 0.02 * v, 0.0])
        p = (K @ (R @ X.T + t[:, None])).T
        uv = p[:, :2] / p[:, 2:] + rng.normal(0, 0.4, (n_pts, 2))
        perm = rng.permutation(n_pts)       # feature k of view v is point perm[k]
        kp = np.zeros((n_pts, 4), np.float32)
        kp[:, :2] = uv[perm]
        kp[:, 2] = 2.0
        write_feat(d / f"v{v}.feat", kp)
        perms.append(perm)
        kps.append(kp)
    pairs, counts, ii, jj = [], [], [], []
    for a in range(n_views):
        inv_b = None
        for b in range(a + 1, n_views):
            inv_b = np.argsort(perms[b])
            m = [(i, int(inv_b[perms[a][i]])) for i in range(n_pts)]
            bad = rng.random(n_pts) < 0.25
            m = [(i, int(rng.integers(n_pts)) if bad[i] else jb) for i, jb in m]
            m.sort()
            pairs.append((a, b))
            counts.append(len(m))
            ii += [x for x, _ in m]
            jj += [y for _, y in m]
    off = np.concatenate([[0], np.cumsum(counts)])
    api.mvg_save_matches(str(d / "matches.putative.bin"),
                         {p: np.stack([ii[off[q]:off[q + 1]], jj[off[q]:off[q + 1]]], 1) for q, p in enumerate(pairs)})
    return pairs, counts, np.array(ii), np.array(jj), kps


@pytest.mark.gpu
def test_filter_stage_gpu(tmp_path, ctx):
    pairs, counts, ii, jj, kps = _stage(tmp_path)
    st = api.sparse_filter(ctx, str(tmp_path))
    assert st.n_pairs_in == len(pairs) and st.n_matches_in == len(ii)
    # expected: the oracle on the same float32 feature positions
    xs, off = [], np.concatenate([[0], np.cumsum(counts)])
    for q, (a, b) in enumerate(pairs):
        k = slice(off[q], off[q + 1])
        xs.append(np.concatenate([kps[a][ii[k], :2], kps[b][jj[k], :2]], 1).astype(np.float64))
    want = oracle_fmatrix_ac(xs, [(640, 480, 640, 480)] * len(pairs))
    got = api.mvg_load_matches(str(tmp_path / "matches.f.bin"))
    kept = [q for q in range(len(pairs)) if want[q]["n_inliers"] > 0]
    assert len(kept) >= len(pairs) - 1
    assert list(got) == [pairs[q] for q in kept]
    for q in kept:
        exp = np.stack([ii[off[q]:off[q + 1]][want[q]["inliers"]], jj[off[q]:off[q + 1]][want[q]["inliers"]]], 1)
        assert np.array_equal(got[pairs[q]], exp)
    assert st.n_pairs_out == len(kept) and st.n_matches_out == sum(want[q]["n_inliers"] for q in kept)


@pytest.mark.gpu
def test_gpu_fmatrix_kernel_timing_opt_in(ctx):
    # the filter's production path takes no events and no extra stream sync:
    # only a context created with SFM_CTX_TIME_KERNELS reports the kernel time
    xs, whs = _batch([(300, 0.2), (800, 0.1)], seed0=900)
    lib = abi.load()
    ms = C.c_double(0.0)
    got = api.fmatrix_ac(ctx, xs, whs)
    assert lib.sfm_ctx_last_kernel_ms(ctx.h, C.byref(ms)) == 0 and ms.value == -1.0
    tctx = api.Context(0, flags=abi.SFM_CTX_TIME_KERNELS)
    try:
        timed = api.fmatrix_ac(tctx, xs, whs)
        assert lib.sfm_ctx_last_kernel_ms(tctx.h, C.byref(ms)) == 0 and ms.value > 0.0
    finally:
        tctx.close()
    for g, t in zip(got, timed):
        _same(g, t)
