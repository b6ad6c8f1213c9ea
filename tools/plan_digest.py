"""Planner refactor check: print the plan digests (SFM_PLAN_DIGEST) and the
planning time of a fixed set of synthetic problems for one library build.

    python tools/plan_digest.py [--lib path/to/libsfmcore.so] [dump.bin ...]

Run it for the old and the new build and diff the outputs (digest lines must
be identical; times are informational).  CPU only (sfm_ba_describe).
"""
import argparse
import ctypes as C
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))

CASES = [
    # (n_cam, n_pt, k, vis_mode, n_intr, model, worlds)
    (20, 2000, 5, 0, 1, 0, (1, 2)),
    (30, 3000, 6, 1, 1, 0, (1, 2)),
    (40, 4000, 6, 2, 1, 0, (1,)),
    (60, 12000, 8, 0, 3, 0, (1, 2, 8)),
    (50, 5000, 7, 1, 5, 0, (1,)),
    (30, 3000, 6, 1, 2, 2, (1,)),
    (80, 8000, 10, 0, 1, 0, (1, 8)),
    (120, 20000, 8, 2, 1, 0, (1,)),
    (300, 30000, 10, 1, 1, 0, (1,)),
    (1000, 500000, 10, 0, 1, 0, (1, 8)),
]


def child(args):
    import numpy as np
    import _helpers as H
    from importlib import import_module
    abi = import_module("3dreconstruction_amd._abi")
    lib = abi.load(args.lib)
    probs = []
    for (n_cam, n_pt, k, vis, n_intr, model, worlds) in CASES:
        sc = H.Scene(n_cam, n_pt, k, vis_mode=vis, n_intr=n_intr, model=model, seed=n_cam * 7 + vis)
        probs.append((f"scene {n_cam}/{n_pt}/{k}/v{vis}/i{n_intr}/m{model}", sc.problem(), worlds, sc))
    sys.path.insert(0, HERE)
    from plan_replay import load_dump, problem
    for path in args.dumps:
        d = load_dump(path)
        probs.append((os.path.basename(path), problem(d), (1,), d))
    for name, pr, worlds, _keep in probs:
        for w in worlds:
            for r in sorted({0, w - 1}):
                shape = abi.BAPlanShape()
                sys.stderr.flush()
                t0 = time.perf_counter()
                rc = lib.sfm_ba_describe(C.byref(pr), r, w, C.byref(shape))
                dt = time.perf_counter() - t0
                assert rc == 0, lib.sfm_last_error()
                print(f"[case] {name} rank {r}/{w}: targets {shape.n_targets} terms {shape.n_terms} "
                      f"pterms {shape.n_pterms} dense {shape.dense} | {dt * 1e3:.1f} ms", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("dumps", nargs="*")
    a = ap.parse_args()
    if a.child:
        child(a)
        return
    env = dict(os.environ, SFM_PLAN_DIGEST="1")
    cmd = [sys.executable, os.path.abspath(__file__), "--child"] + (["--lib", a.lib] if a.lib else []) + a.dumps
    r = subprocess.run(cmd, env=env, stderr=subprocess.PIPE, text=True)
    for line in r.stderr.splitlines():
        print(line)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
