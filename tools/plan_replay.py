"""Replay the BA planner on problems dumped by the C5 loop (SFM_SEQ_DUMP).

    python tools/plan_replay.py <dump.bin> [...] [--reps N]

Runs the host planner (sfm_ba_describe, no GPU) on each dump, prints the
plan's shape and the best wall time over the repetitions; with SFM_TIMING=1
in the environment the planner's phase lines go to stderr.
"""
import argparse
import ctypes as C
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
abi = importlib.import_module("3dreconstruction_amd._abi")


def load_dump(path):
    raw = open(path, "rb").read()
    n_img, n_intr, n_pt, n_obs, const_img = np.frombuffer(raw, np.int64, 5)
    o = 40
    pt_off = np.frombuffer(raw, np.int64, n_pt + 1, o); o += 8 * (n_pt + 1)
    obs_img = np.frombuffer(raw, np.int32, n_obs, o); o += 4 * n_obs
    obs_uv = np.frombuffer(raw, np.float64, 2 * n_obs, o); o += 16 * n_obs
    img_intr = np.frombuffer(raw, np.int32, n_img, o)
    return dict(n_img=int(n_img), n_intr=int(n_intr), n_pt=int(n_pt), n_obs=int(n_obs),
                const_img=int(const_img), pt_offsets=pt_off.copy(), obs_img=obs_img.copy(),
                obs_uv=obs_uv.copy(), img_intr=img_intr.copy())


def problem(d, model=0):
    p = abi.BAProblem()
    p.n_img, p.n_intr, p.n_pt, p.n_obs = d["n_img"], d["n_intr"], d["n_pt"], d["n_obs"]
    p.pt_offsets = d["pt_offsets"].ctypes.data_as(abi.i64p)
    p.obs_img = d["obs_img"].ctypes.data_as(abi.i32p)
    p.obs_uv = d["obs_uv"].ctypes.data_as(abi.f64p)
    p.img_intr = d["img_intr"].ctypes.data_as(abi.i32p)
    p.const_img = d["const_img"]
    p.camera_model = model
    p.huber_a = 4.0
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dumps", nargs="+")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    lib = abi.load()
    for path in a.dumps:
        d = load_dump(path)
        p = problem(d)
        shape = abi.BAPlanShape()
        best = 1e30
        for _ in range(a.reps):
            t0 = time.perf_counter()
            rc = lib.sfm_ba_describe(C.byref(p), 0, 1, C.byref(shape))
            best = min(best, time.perf_counter() - t0)
            assert rc == 0, lib.sfm_last_error()
        print(f"{os.path.basename(path)}: img {d['n_img']} pt {d['n_pt']} obs {d['n_obs']} | "
              f"dense {shape.dense} D {shape.band_blocks} chunks {shape.n_chunks} cpt {shape.n_chunk_pts} "
              f"gpt {shape.n_general_pts} targets {shape.n_targets} terms {shape.n_terms} "
              f"pterms {shape.n_pterms} | plan {best * 1e3:.2f} ms")


if __name__ == "__main__":
    main()
