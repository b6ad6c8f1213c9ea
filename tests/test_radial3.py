"""OpenMVG's PINHOLE_CAMERA_RADIAL3 residual with ADJUST_ALL, the model
sparseBuilder::reconstruction() selects (src/sparseBuilder/sparseBuilder.cpp:
1292-1299; OpenMVG ResidualErrorFunctor_Pinhole_Intrinsic_Radial_K3; SURVEY.md
§8(f) row 4), selected by sfm_ba_problem.camera_model = SFM_CAM_RADIAL3 with
6-double intrinsics blocks {f, ppx, ppy, k1, k2, k3}.

OpenMVG is not vendored in /root/reference, so the functor is restated from
its published form (parity unpinned beyond the restatement): the oracle's
analytic Jacobian is checked against dual numbers run through a term-by-term
restatement of the functor (the Ceres AutoDiff path) and against finite
differences; noise-free scenes recover the ground truth.
GPU: the HIP path against the oracle with the same bars as the pinhole model:
banded sequences on the Schur chunk tiles (6-row intrinsics slots, 80-row
tiles) and block cyclic reduction with a 6-column-per-block arrow; random
visibility, long tracks or many intrinsics blocks on the general-point path and
the dense reduced camera system.
"""
import importlib

import numpy as np
import pytest

import _helpers as H

abi = H.abi
api = importlib.import_module("3dreconstruction_amd.api")
R3 = abi.SFM_CAM_RADIAL3


def _jac(mode, intr, extr, X, uv):
    r = np.zeros(2)
    J = np.zeros(30)
    rc = H.oracle().orc_ba_jacobian_model(R3, mode, abi.ptr(intr, abi.f64p), abi.ptr(extr, abi.f64p),
                                          abi.ptr(X, abi.f64p), abi.ptr(uv, abi.f64p),
                                          abi.ptr(r, abi.f64p), abi.ptr(J, abi.f64p))
    assert rc == 0
    return r, J.reshape(2, 15)


def _point(rng, log_theta):
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    extr = np.concatenate([axis * 10 ** log_theta, rng.normal(size=3) * 0.3 + [0, 0, 9]])
    intr = np.array([2900.0, 1416.0, 1064.0, -0.05, 0.01, -0.002]) * (1 + 0.1 * rng.normal(size=6))
    return intr, extr, rng.normal(size=3), rng.normal(size=2) * 200 + [1416, 1064]


def test_intr_width():
    lib = abi.load()
    assert [lib.sfm_ba_intr_width(m) for m in (0, 1, 2, 3, -1)] == [4, 4, 6, 0, 0]


@pytest.mark.parametrize("log_theta", [-12, -7, -1, 0.4])
def test_radial3_jacobian_vs_autodiff(log_theta):
    rng = np.random.default_rng(int(abs(log_theta) * 10) + 7)
    for _ in range(20):
        intr, extr, X, uv = _point(rng, log_theta)
        r0, J0 = _jac(0, intr, extr, X, uv)
        r1, J1 = _jac(1, intr, extr, X, uv)
        np.testing.assert_allclose(r0, r1, rtol=1e-13, atol=1e-9)
        np.testing.assert_allclose(J0, J1, rtol=1e-9, atol=1e-9 * np.abs(J1).max())
        # d r_x / d ppx = 1, d r_x / d ppy = 0 (and the mirror for r_y)
        assert J0[0, 1] == 1.0 and J0[0, 2] == 0.0 and J0[1, 1] == 0.0 and J0[1, 2] == 1.0


def test_radial3_jacobian_vs_finite_differences():
    rng = np.random.default_rng(9)
    for _ in range(10):
        intr, extr, X, uv = _point(rng, -1)
        _, J = _jac(0, intr, extr, X, uv)
        theta = np.concatenate([intr, extr, X])
        for k in range(15):
            h = 1e-6 * max(1.0, abs(theta[k]))
            tp, tm = theta.copy(), theta.copy()
            tp[k] += h
            tm[k] -= h
            rp, _ = _jac(0, tp[:6], tp[6:12], tp[12:], uv)
            rm, _ = _jac(0, tm[:6], tm[6:12], tm[12:], uv)
            np.testing.assert_allclose(J[:, k], (rp - rm) / (2 * h), rtol=2e-5,
                                       atol=2e-5 * (np.abs(J).max() + 1))


def test_radial3_synth_projects_with_the_functor():
    # noise-free observations of the synthetic scene are zero-residual under
    # the oracle's restatement at the ground truth
    sc = H.Scene(12, 300, 4, model=R3, noise=0.0, outliers=0.0)
    assert sc.intr.shape == (6,)
    cost = H.oracle_cost(sc, sc.gt_extr, sc.gt_intr, sc.gt_X)
    assert cost < 1e-18


def test_radial3_noise_free_recovers_ground_truth():
    sc = H.Scene(20, 2000, 4, model=R3, noise=0.0, outliers=0.0)
    rc, s, _, (e, i, x) = H.oracle_solve(sc)
    assert rc == 0 and s.usable
    assert s.final_cost < 1e-10 * s.initial_cost
    np.testing.assert_allclose(i[[0, 3, 4]], sc.gt_intr[[0, 3, 4]], rtol=1e-5, atol=1e-7)


def _shape(sc):
    shp = abi.BAPlanShape()
    assert abi.load().sfm_ba_describe(H.C.byref(sc.problem()), 0, 1, H.C.byref(shp)) == 0
    return shp


def test_radial3_planner_shape():
    # a banded sequence: every point on the chunk tiles (6 rows per camera,
    # 6 per intrinsics block: 80-row tiles), the band + arrow RCS, 6 columns
    # per intrinsics block
    sc = H.Scene(24, 3000, 6, model=R3, n_intr=2, seed=5)
    shp = _shape(sc)
    assert shp.n_chunks > 0 and shp.n_chunk_pts == sc.n_pt and shp.n_general_pts == 0
    assert shp.dense == 0 and shp.rcs_dim == 6 * (sc.n_cam - 1) + 6 * 2
    # the arrow holds at most 16 bordered columns: three 6-wide blocks are dense
    sc3 = H.Scene(24, 3000, 6, model=R3, n_intr=3, seed=5)
    shp3 = _shape(sc3)
    assert shp3.dense == 1 and shp3.n_chunk_pts == sc3.n_pt
    # random visibility: general points and a dense RCS, as for pinhole
    scr = H.Scene(30, 1200, 6, vis_mode=1, model=R3, seed=3)
    shpr = _shape(scr)
    assert shpr.dense == 1 and shpr.n_general_pts > 0


# ---------------------------------------------------------------------------
# GPU parity (HIP path through the C-ABI vs the oracle)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = api.Context(0)
    yield c
    c.close()


def _compare(ctx, sc, rtol=1e-6):
    orc_rc, os_, otr, (oe, oi, ox) = H.oracle_solve(sc, threads=8)
    e, i, x = sc.params()
    plan = api.BAPlan(ctx, sc.problem(), e, i, x)
    rc, gs = plan.run(check=False)
    gtr = plan.trace()
    e, i, x = plan.download()
    plan.close()
    assert rc == orc_rc == 0
    assert (gs.termination, gs.iterations, gs.successful_steps) == \
           (os_.termination, os_.iterations, os_.successful_steps)
    assert len(gtr) == len(otr)
    for g, o in zip(gtr, otr):
        assert (g.step_is_valid, g.step_is_successful) == (o.step_is_valid, o.step_is_successful)
        assert abs(g.cost / o.cost - 1) < 1e-9
    assert abs(gs.initial_cost / os_.initial_cost - 1) < 1e-12
    assert abs(gs.rmse_final / os_.rmse_final - 1) < rtol
    np.testing.assert_allclose(i[0::6], oi[0::6], rtol=1e-3)
    assert abs(H.oracle_cost(sc, e, i, x) / gs.final_cost - 1) < 1e-9
    return gs, os_, (e, i, x)


@pytest.mark.gpu
def test_radial3_gpu_c1(ctx):
    sc = H.Scene(20, 2000, 4, model=R3)
    gs, _, _ = _compare(ctx, sc)
    assert gs.final_cost < 0.1 * gs.initial_cost


@pytest.mark.gpu
@pytest.mark.parametrize("args", [dict(n_cam=24, n_pt=3000, k=8, seed=17),
                                  dict(n_cam=16, n_pt=1500, k=5, n_intr=3, seed=11),
                                  dict(n_cam=30, n_pt=1200, k=6, vis_mode=1, seed=3),
                                  dict(n_cam=12, n_pt=800, k=12, n_intr=12, seed=29)])
def test_radial3_gpu_shapes(ctx, args):
    _compare(ctx, H.Scene(model=R3, **args))


@pytest.mark.gpu
def test_radial3_gpu_c2(ctx):
    sc = H.Scene(200, 50_000, 10, model=R3, seed=0x5F3D0002)
    assert _shape(sc).dense == 0 and _shape(sc).n_chunk_pts == sc.n_pt   # chunk tiles + BCR
    _compare(ctx, sc)


@pytest.mark.gpu
def test_radial3_band_equals_dense_solver(ctx):
    # the chunk + BCR path and the general + dense path solve the same system
    sc = H.Scene(40, 5000, 8, model=R3, n_intr=2, seed=41)
    res = []
    for dense in (False, True):
        with H.engine_ctx(H.abi.SFM_CTX_BA_DENSE_RCS if dense else 0) as c:
            plan = api.BAPlan(c, sc.problem(), *sc.params())
            _, s = plan.run()
            res.append((s, plan.trace()))
            plan.close()
    (s0, t0), (s1, t1) = res
    assert s0.iterations == s1.iterations
    assert abs(s0.final_cost / s1.final_cost - 1) < 1e-9
    for a, b in zip(t0, t1):
        assert a.step_is_successful == b.step_is_successful


def test_radial3_regression_pin_c1():
    # the oracle's C1 trajectory under RADIAL3 (tests/golden/make_golden.py
    # --ba-only regenerates it; the pinhole and Snavely pins came out
    # byte-identical after the 6-wide intrinsics generalisation of the oracle)
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ba_c1_radial3_oracle.json")))
    sc = H.Scene(g["scene"]["n_cam"], g["scene"]["n_pt"], g["scene"]["k"], seed=g["scene"]["seed"], model=R3)
    rc, s, tr, _ = H.oracle_solve(sc, threads=1)
    assert rc == g["rc"] and s.iterations == g["iterations"]
    assert s.successful_steps == g["successful_steps"]
    assert abs(s.final_cost / g["final_cost"] - 1) < 1e-9
    for t, gt in zip(tr, g["trace"]):
        assert [t.iteration, t.step_is_valid, t.step_is_successful] == gt[:3]
        assert abs(t.cost / gt[3] - 1) < 1e-9
