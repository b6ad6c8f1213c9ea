#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ (run in the build container).

Matching fixtures: RootSIFT uchar descriptors produced by the reference's own
in-tree VLFeat (src/nonFree/sift/vl, built by oracle/build_ref.sh into
oracle/_ref/) on three deterministic synthetic views, plus the expected match
lists for every pair in both modes.  Expected outputs come from an
independent numpy brute force, and the script asserts that the oracle
(oracle/match_oracle.cpp) agrees before writing anything.

BA fixture: the oracle's summary and iteration trace on a small deterministic
scene (a regression pin of the restatement; Ceres itself is unavailable, so
this is not a reference output).
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _helpers as H  # noqa: E402

TOOL = os.path.join(ROOT, "oracle", "_ref", "vlsift_tool")
VIEWS = [  # seed, angle, tx, ty, scale  (same scene, three viewpoints)
    (7, 0.0, 0.0, 0.0, 1.0),
    (7, 0.2, 12.0, -7.0, 1.1),
    (7, -0.35, -20.0, 15.0, 0.9),
]
R2 = np.float32(np.float32(0.8) * np.float32(0.8))


def numpy_match(a, b, mode):
    a = a.astype(np.int64)
    b = b.astype(np.int64)
    D = (a * a).sum(1)[:, None] + (b * b).sum(1)[None, :] - 2 * a @ b.T   # [|a|, |b|]
    if mode == 0:   # queries = rows of b, database = rows of a
        if len(a) < 2 or len(b) == 0:
            return np.full(len(b), -1), np.full(len(b), -1)
        nn = np.argmin(D, axis=0)           # first minimum = lowest index
        d1 = D[nn, np.arange(len(b))]
        if len(a) < 2:
            return np.full(len(b), -1), np.full(len(b), -1)
        d2 = np.partition(D, 1, axis=0)[1]
        keep = np.float32(d1) < R2 * np.float32(d2)
        return np.where(keep, nn, -1), np.where(keep, d1, -1)
    if len(a) == 0 or len(b) == 0:
        return np.full(len(a), -1), np.full(len(a), -1)
    nq = np.argmin(D, axis=1)
    nt = np.argmin(D, axis=0)
    keep = nt[nq] == np.arange(len(a))
    return np.where(keep, nq, -1), np.where(keep, D[np.arange(len(a)), nq], -1)


def main():
    if not os.path.exists(TOOL):
        subprocess.run(["bash", os.path.join(ROOT, "oracle", "build_ref.sh")], check=True)
    desc = []
    for k, (seed, ang, tx, ty, sc) in enumerate(VIEWS):
        u8 = os.path.join(HERE, f"vlfeat_view{k}.u8")
        kp = os.path.join(HERE, f"vlfeat_view{k}.kp")
        subprocess.run([TOOL, u8, kp, "640", "480", str(seed), str(ang), str(tx), str(ty), str(sc)],
                       check=True, capture_output=True)
        desc.append(np.fromfile(u8, np.uint8).reshape(-1, 128))
    expected = {"views": [len(d) for d in desc], "pairs": {}}
    for i in range(len(desc)):
        for j in range(len(desc)):
            if i == j:
                continue
            for mode in (0, 1):
                ni, nd = numpy_match(desc[i], desc[j], mode)
                oi, od = H.oracle_match_dense(desc[i], desc[j], mode)
                assert np.array_equal(ni, oi) and np.array_equal(nd, od), (i, j, mode)
                expected["pairs"][f"{i}-{j}-{mode}"] = {"idx": ni.tolist(), "d2": nd.tolist()}
    with open(os.path.join(HERE, "vlfeat_matches.json"), "w") as f:
        json.dump(expected, f)

    n = write_ba_pins()
    print("golden fixtures written:", expected["views"], "BA iterations", n)


def write_ba_pin(name, model):
    """Oracle trajectory of the C1 scene (20 cams / 2000 pts / k 4), one thread."""
    sc = H.Scene(20, 2000, 4, seed=0x5F3D0001, model=model)
    rc, s, tr, (e, i, x) = H.oracle_solve(sc)
    ba = {"scene": {"n_cam": 20, "n_pt": 2000, "k": 4, "seed": 0x5F3D0001, "camera_model": model},
          "rc": rc, "iterations": s.iterations, "successful_steps": s.successful_steps,
          "unsuccessful_steps": s.unsuccessful_steps, "termination": s.termination,
          "initial_cost": s.initial_cost, "final_cost": s.final_cost,
          "rmse_initial": s.rmse_initial, "rmse_final": s.rmse_final,
          "trace": [[t.iteration, t.step_is_valid, t.step_is_successful, t.cost,
                     t.trust_region_radius] for t in tr]}
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(ba, f, indent=1)
    return s.iterations


def write_ba_pins():
    n = write_ba_pin("ba_c1_oracle.json", 0)
    write_ba_pin("ba_c1_snavely_oracle.json", 1)   # SnavelyReprojectionError.h model
    write_ba_pin("ba_c1_radial3_oracle.json", 2)   # OpenMVG PINHOLE_CAMERA_RADIAL3
    return n


if __name__ == "__main__":
    if "--ba-only" in sys.argv:   # trajectories only (no VLFeat rebuild)
        write_ba_pins()
    else:
        main()
