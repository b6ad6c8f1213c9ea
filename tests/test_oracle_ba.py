"""CPU: the BA oracle — analytic Jacobian vs dual numbers (the Ceres AutoDiff
path) and finite differences, Huber branch, convergence on noise-free
scenes, and the regression pin tests/golden/ba_c1_oracle.json."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import _helpers as H

abi = H.abi
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _jac(mode, intr, extr, X, uv):
    r = np.zeros(2)
    J = np.zeros(26)
    rc = H.oracle().orc_ba_jacobian(mode, abi.ptr(intr, abi.f64p), abi.ptr(extr, abi.f64p),
                                    abi.ptr(X, abi.f64p), abi.ptr(uv, abi.f64p),
                                    abi.ptr(r, abi.f64p), abi.ptr(J, abi.f64p))
    assert rc == 0
    return r, J.reshape(2, 13)


@pytest.mark.parametrize("log_theta", [-12, -8.5, -7, -4, -1, 0.3, 0.5])
def test_jacobian_analytic_vs_autodiff(log_theta):
    rng = np.random.default_rng(int(abs(log_theta) * 10))
    for _ in range(20):
        axis = rng.normal(size=3)
        axis /= np.linalg.norm(axis)
        w = axis * 10 ** log_theta
        extr = np.concatenate([w, rng.normal(size=3) * 0.3 + [0, 0, 9]])
        intr = np.array([2905.88, 2903.1, 1416.0, 1064.0])
        X = rng.normal(size=3)
        uv = np.array([1400.0, 1050.0])
        r0, J0 = _jac(0, intr, extr, X, uv)
        r1, J1 = _jac(1, intr, extr, X, uv)
        np.testing.assert_allclose(r0, r1, rtol=1e-14, atol=1e-12)  # Jet a/b = a*(1/b)
        tol = 1e-7 if log_theta > -8 else 1e-5  # G&Y formula loses ~eps/theta near 0
        assert np.abs(J0 - J1).max() <= tol * max(1.0, np.abs(J1).max())


def test_jacobian_vs_finite_differences():
    rng = np.random.default_rng(3)
    intr = np.array([2905.88, 2905.88, 1416.0, 1064.0])
    for _ in range(10):
        extr = np.concatenate([rng.normal(size=3) * 0.5, [0.1, -0.2, 10.0]])
        X = rng.normal(size=3)
        uv = np.array([1300.0, 1100.0])
        _, J = _jac(0, intr, extr, X, uv)
        params = [intr, extr, X]
        col = 0
        for blk in params:
            for a in range(len(blk)):
                h = 1e-6 * max(1.0, abs(blk[a]))
                p = [q.copy() for q in params]
                m = [q.copy() for q in params]
                p[params.index(blk) if False else [id(q) for q in params].index(id(blk))][a] += h
                m[[id(q) for q in params].index(id(blk))][a] -= h
                rp, _ = _jac(0, *p, uv)
                rm, _ = _jac(0, *m, uv)
                fd = (rp - rm) / (2 * h)
                assert np.abs(fd - J[:, col]).max() < 1e-4 * max(1.0, np.abs(J[:, col]).max())
                col += 1


def test_huber_branch_switch():
    sc = H.Scene(6, 50, 3, noise=0.0, outliers=0.0, perturb=(0, 0, 0, 0))
    e, i, x = sc.params()
    res = np.zeros(2 * sc.n_obs)
    c = C.c_double()
    # move one observation by 3 px (inlier, rho = s) and one by 5 px (outlier)
    sc.obs_uv[0] += 3.0
    sc.obs_uv[2] += 5.0
    H.oracle().orc_ba_cost(C.byref(sc.problem()), abi.ptr(e, abi.f64p), abi.ptr(i, abi.f64p),
                           abi.ptr(x, abi.f64p), C.byref(c), abi.ptr(res, abi.f64p))
    r = res.reshape(-1, 2)
    s0 = (r[0] ** 2).sum()
    s1 = (r[1] ** 2).sum()
    rest = 0.5 * (r[2:] ** 2).sum()
    assert s0 < 16 < s1
    expect = 0.5 * s0 + 0.5 * (2 * 4 * np.sqrt(s1) - 16) + rest
    assert abs(c.value - expect) < 1e-9 * max(1, expect)


def test_noise_free_convergence():
    sc = H.Scene(10, 500, 4, noise=0.0, outliers=0.0)
    rc, s, tr, (e, i, x) = H.oracle_solve(sc)
    assert rc == 0 and s.usable
    assert s.final_cost < 1e-10 * s.initial_cost
    np.testing.assert_allclose(i, sc.gt_intr, rtol=1e-6)


def test_regression_pin_c1():
    g = json.load(open(os.path.join(GOLD, "ba_c1_oracle.json")))
    sc = H.Scene(g["scene"]["n_cam"], g["scene"]["n_pt"], g["scene"]["k"], seed=g["scene"]["seed"])
    # single thread: the summation order (and, at the function-tolerance
    # boundary, the iteration count) is that of the generating run
    rc, s, tr, _ = H.oracle_solve(sc, threads=1)
    assert rc == g["rc"] and s.iterations == g["iterations"]
    assert s.successful_steps == g["successful_steps"]
    assert abs(s.final_cost / g["final_cost"] - 1) < 1e-9
    for t, gt in zip(tr, g["trace"]):
        assert [t.iteration, t.step_is_valid, t.step_is_successful] == gt[:3]
        assert abs(t.cost / gt[3] - 1) < 1e-9


def test_thread_count_invariance():
    sc = H.Scene(20, 1500, 5, seed=77)
    _, s1, _, r1 = H.oracle_solve(sc, threads=1)
    _, s4, _, r4 = H.oracle_solve(sc, threads=4)
    # summation order differs; termination (|dcost| <= 1e-6 cost) may move by
    # one iteration, which moves the final cost by at most ~1e-6 relative
    assert abs(s1.iterations - s4.iterations) <= 1
    assert abs(s1.final_cost / s4.final_cost - 1) < 2e-6


def test_gauge_image_untouched_and_failure_semantics():
    sc = H.Scene(8, 200, 3, seed=4)
    rc, s, tr, (e, i, x) = H.oracle_solve(sc)
    np.testing.assert_array_equal(e[6:12], sc.extr[6:12])   # const_img = 1
    sc.X[0] = np.nan
    rc, s, tr, (e2, i2, x2) = H.oracle_solve(sc)
    assert rc == abi.SFM_ERR_NOT_FINITE and not s.usable
    np.testing.assert_array_equal(e2, sc.extr)               # world left untouched
