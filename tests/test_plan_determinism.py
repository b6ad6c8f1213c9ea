"""The host planner's output does not depend on how its phases are split over
host threads (ba_plan.cpp: the counting-scatter reduce plan takes rows in
ranges of equal work, the chunker fixed point ranges): every plan array's
digest (SFM_PLAN_DIGEST, sfm_ba_describe) is the same with 1, 3 and 8
planner threads, for band, dense, arrow, RADIAL3 and sharded plans.  CPU only."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

CHILD = r"""
import sys, ctypes as C, importlib
sys.path.insert(0, %r); sys.path.insert(0, %r)
import _helpers as H
abi = importlib.import_module("3dreconstruction_amd._abi")
lib = abi.load()
cases = [(40, 4000, 6, 0, 1, 0, 1), (40, 4000, 6, 1, 1, 0, 1), (60, 12000, 8, 0, 3, 0, 2),
         (30, 3000, 6, 1, 2, 2, 1), (120, 20000, 8, 2, 1, 0, 1), (80, 8000, 10, 0, 1, 0, 8)]
for (n_cam, n_pt, k, vis, n_intr, model, world) in cases:
    sc = H.Scene(n_cam, n_pt, k, vis_mode=vis, n_intr=n_intr, model=model, seed=n_cam + vis)
    pr = sc.problem()
    for r in range(world):
        sh = abi.BAPlanShape()
        assert lib.sfm_ba_describe(C.byref(pr), r, world, C.byref(sh)) == 0, lib.sfm_last_error()
"""


def _digests(threads):
    env = dict(os.environ, SFM_PLAN_DIGEST="1", SFM_PLAN_THREADS=str(threads))
    r = subprocess.run([sys.executable, "-c", CHILD % (HERE, ROOT)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stderr.splitlines() if ln.startswith("[digest]")]
    assert len(lines) == 14
    return lines


def test_plan_independent_of_planner_threads():
    one = _digests(1)
    assert _digests(3) == one
    assert _digests(8) == one
