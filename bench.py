#!/usr/bin/env python3
"""Benchmark: BA LM-iterations/s (+ obs/s) on the C4 scene and all-pairs SIFT
matching pairs/s on the C3 collection (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W

A step is one complete bundle adjustment (sfm_ba_plan_run: Ceres-semantics LM
from the same initial point to termination) of the C4 scene — 1000 cameras,
500k points, 5M observations, banded orbit visibility k=10, Huber(4), gauge
camera 1 — with all inputs resident in HBM.  value = LM iterations completed by
the whole job / wall time (max over ranks).  For N>1 every rank holds one
landmark block and the reduced camera system is all-reduced over RCCL inside
libsfmcore (strong scaling: the problem is fixed).

The C3 matcher (500 frames x 4096 x 128-D uint8, exhaustive 124,750 pairs,
ratio 0.8) runs after the BA steps; pairs are split across ranks.

cpu_baseline: the oracle (test infrastructure, CPU restatement of the
reference Ceres semantics) on a bounded sample, rank 0 at N=1 only.
"""
import argparse
import ctypes as C
import importlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def _requested_gpus(argv):
    for k, a in enumerate(argv):
        if a == "--gpus" and k + 1 < len(argv):
            return int(argv[k + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return 1


def _self_launch(n):
    """`bench.py --gpus N` outside a launcher: start N ranks (one process per
    GPU) through torch.distributed.run as a CHILD process and exit with its
    code.  Runs before anything in this process loads HIP or touches a GPU."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    print(f"[bench] launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


if __name__ == "__main__" and "WORLD_SIZE" not in os.environ and "--pmc-child" not in sys.argv:
    _n = _requested_gpus(sys.argv[1:])
    if _n > 1:
        sys.exit(_self_launch(_n))

import numpy as np  # noqa: E402

sys.path.insert(0, ROOT)
abi = importlib.import_module("3dreconstruction_amd._abi")
api = importlib.import_module("3dreconstruction_amd.api")

FP64_PEAK_TF = 78.6     # MI355X dense FP64 (vector = matrix), TFLOP/s
I8_PEAK_TOPS = 5000.0   # MI355X dense int8 MFMA = 2x bf16 (2.5 PF), TOP/s
HBM_PEAK_GBS = 8000.0


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def c4_scene(n_cam=1000, n_pt=500_000, k=10, seed=0x5F3D0004, model=0, vis=0, n_intr=1):
    lib = abi.load()
    cfg = abi.SynthBAConfig()
    cfg.camera_model = model
    cfg.n_cam, cfg.k, cfg.vis_mode, cfg.n_intr = n_cam, k, vis, n_intr
    cfg.n_pt, cfg.seed = n_pt, seed
    cfg.noise_px, cfg.outlier_frac = 0.5, 0.01
    cfg.perturb_rot, cfg.perturb_t, cfg.perturb_X, cfg.perturb_f = 0.01, 0.05, 0.05, 5.0
    cfg.const_img = 1
    n_obs = C.c_int64()
    lib.sfm_synth_ba(C.byref(cfg), None, None, None, None, None, None, None, None, None, None,
                     C.byref(n_obs))
    no = n_obs.value
    sc = {
        "pt_offsets": np.zeros(n_pt + 1, np.int64), "obs_img": np.zeros(no, np.int32),
        "obs_uv": np.zeros(2 * no), "img_intr": np.zeros(n_cam, np.int32),
        "extr": np.zeros(6 * n_cam), "intr": np.zeros(lib.sfm_ba_intr_width(model) * n_intr), "X": np.zeros(3 * n_pt),
    }
    p = abi.ptr
    rc = lib.sfm_synth_ba(C.byref(cfg), p(sc["pt_offsets"], abi.i64p), p(sc["obs_img"], abi.i32p),
                          p(sc["obs_uv"], abi.f64p), p(sc["img_intr"], abi.i32p),
                          p(sc["extr"], abi.f64p), p(sc["intr"], abi.f64p), p(sc["X"], abi.f64p),
                          None, None, None, C.byref(n_obs))
    assert rc == 0
    pr = abi.BAProblem()
    pr.n_img, pr.n_intr, pr.n_pt, pr.n_obs = n_cam, n_intr, n_pt, no
    pr.pt_offsets = p(sc["pt_offsets"], abi.i64p)
    pr.obs_img = p(sc["obs_img"], abi.i32p)
    pr.obs_uv = p(sc["obs_uv"], abi.f64p)
    pr.img_intr = p(sc["img_intr"], abi.i32p)
    pr.const_img = 1
    pr.camera_model = model
    pr.huber_a = 4.0
    sc["problem"] = pr
    sc["n_obs"] = no
    return sc


def host_cpu():
    """CPU model and the thread budget of this process (OMP_NUM_THREADS on the
    GPU box is this GPU's share of the host)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    n = os.cpu_count() or 1
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return model, max(1, min(n, 64))


def cpu_baseline_ba(sc):
    """Oracle (CPU restatement of the reference Ceres semantics) on the same C4
    scene: a full solve to termination on all of this process's host threads
    (value), and the first LM iterations on one thread, as the reference runs
    Ceres (num_threads = 1, BundleAdjuster.h:170)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _helpers as H  # test infrastructure: the oracle is only the baseline here
    lib = H.oracle()
    model, threads = host_cpu()

    def solve(max_iters, nthreads):
        o = abi.default_options()
        o.max_num_iterations = max_iters
        e, i, x = sc["extr"].copy(), sc["intr"].copy(), sc["X"].copy()
        s = abi.BASummary()
        tr = (abi.BAIter * 64)()
        tn = C.c_int32()
        t = time.time()
        lib.orc_ba_solve(C.byref(sc["problem"]), abi.ptr(e, abi.f64p), abi.ptr(i, abi.f64p),
                         abi.ptr(x, abi.f64p), C.byref(o), C.byref(s), tr, 64, C.byref(tn), None, 0,
                         H.ALLREDUCE_FN(), None, nthreads)
        return s, time.time() - t

    s_all, dt_all = solve(50, threads)
    s_one, dt_one = solve(2, 1)
    return {"value": s_all.iterations / dt_all, "unit": "LM-iters/s", "cores": threads, "kind": "port",
            "cpu_model": model,
            "sample": f"C4 scene (1000 cams/500k pts/5M obs), full solve to termination "
                      f"({s_all.iterations} LM iterations incl. iteration-0 linearisation and Jacobi "
                      f"scaling) on {threads} threads, {dt_all:.1f} s wall; oracle = CPU restatement of the "
                      "reference Ceres semantics, not Ceres itself",
            "obs_per_sec": s_all.iterations * sc["n_obs"] / dt_all,
            "rmse_final": s_all.rmse_final,
            "single_thread": {"value": s_one.iterations / dt_one, "unit": "LM-iters/s", "cores": 1,
                              "sample": f"first {s_one.iterations} LM iterations incl. iteration 0, "
                                        f"{dt_one:.1f} s wall (Ceres num_threads = 1)"}}


def cpu_baseline_match(desc, n_kp, pairs, n_pairs=96):
    """The oracle (exact integer brute force) on pairs spread over the whole C3
    list, on all of this process's host threads."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _helpers as H
    lib = H.oracle()
    model, threads = host_cpu()
    off = np.arange(desc.shape[0] // n_kp + 1, dtype=np.int64) * n_kp
    pick = np.linspace(0, len(pairs) - 1, n_pairs).astype(np.int64)
    sub = np.ascontiguousarray(pairs[pick])
    counts = np.zeros(n_pairs, np.int64)
    t = time.time()
    lib.orc_match_pairs(abi.ptr(desc, abi.u8p), abi.ptr(off, abi.i64p), len(off) - 1,
                        abi.ptr(sub, abi.i32p), n_pairs, abi.SFM_MATCH_RATIO, 0.8, threads,
                        abi.ptr(counts, abi.i64p), None, None, None)
    dt = time.time() - t
    return {"value": n_pairs / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "cpu_model": model,
            "sample": f"{n_pairs} pairs evenly spaced over the C3 list, exact integer brute force, "
                      f"{dt:.1f} s wall"}


def cpu_baseline_cascade(desc, n_kp, n_img=24):
    """The oracle on every pair among the first n_img images (hashing
    included, so the sample is hashing-heavier than the full list)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _helpers as H
    lib = H.oracle()
    model, threads = host_cpu()
    off = np.arange(desc.shape[0] // n_kp + 1, dtype=np.int64) * n_kp
    sub = np.array([(i, j) for i in range(n_img) for j in range(i + 1, n_img)], np.int32)
    n_pairs = len(sub)
    counts = np.zeros(n_pairs, np.int64)
    t = time.time()
    lib.orc_match_pairs(abi.ptr(desc, abi.u8p), abi.ptr(off, abi.i64p), len(off) - 1,
                        abi.ptr(sub, abi.i32p), n_pairs, abi.SFM_MATCH_CASCADE, 0.8, threads,
                        abi.ptr(counts, abi.i64p), None, None, None)
    dt = time.time() - t
    n_used = len(np.unique(sub))
    return {"value": n_pairs / dt, "unit": "pairs/s", "cores": threads, "kind": "port", "cpu_model": model,
            "sample": f"all {n_pairs} pairs among the first {n_used} C3 images, incl. hashing "
                      f"them, cascade-hashing restatement, {dt:.1f} s wall"}


def pmc_traffic(kernel, largest=False):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc
    summary of this configuration (profiles/r*/pmc_summary.json, written by
    tools/pmc_summary.py: FETCH_SIZE x2 per the gfx950 note + WRITE_SIZE).
    None when no summary is present."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                          "profiles", "r*", "pmc_summary.json")))
    if not files:
        return None
    try:
        ks = json.load(open(files[-1]))["kernels"]
    except Exception:
        return None
    for name, e in ks.items():
        if name.startswith(kernel) and "traffic_bytes" in e:
            return e.get("traffic_bytes_max", e["traffic_bytes"]) if largest else e["traffic_bytes"]
    return None


# rocprofv3 counter passes run by this benchmark on itself (a child process
# per pass, the program directly after `--`).  gfx950 slot limits
# (MI355X_MICROARCH.md §rocprofv3 PMC slots): FETCH_SIZE uses 3 of the 4 TCC
# slots and WRITE_SIZE 2, so they take separate passes.
PMC_PASSES = [["FETCH_SIZE"],
              ["WRITE_SIZE", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"]]


def pmc_child(args):
    """--pmc-child: the C4 plan and two solves, nothing else (profiled by the
    parent's rocprofv3 passes)."""
    ctx = api.Context(0)
    sc = c4_scene(args.n_cam, args.n_pt)
    plan = api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
    for _ in range(2):
        plan.run()
    ctx.synchronize()
    plan.close()
    ctx.close()


def pmc_child_match(args):
    """--pmc-child-match: the C3 collection matched once (ratio mode, every
    pair in one launch, as the bench's timed run), nothing else."""
    ctx = api.Context(0)
    nf, nkp = args.match_frames, 4096
    desc = api.synth_descriptors(nf, nkp)
    off = np.arange(nf + 1, dtype=np.int64) * nkp
    mplan = api.MatchPlan(ctx, desc, off)
    mplan.run(api.exhaustive_pairs(nf), count=False)
    ctx.synchronize()
    mplan.close()
    ctx.close()


def kstats_measure(args, kernel_prefix="schur_kernel<0, 4, 5, 52, false>"):
    """rocprofv3 --kernel-trace --stats over the same child run as the --pmc
    passes (the C4 plan and two solves): mean duration (ms) and launch count
    of the Schur kernel's non-first launches, from the profiler's own summary
    (the profile-backed figure beside the in-run HIP-event
    one).  None when rocprofv3 is unavailable or the pass fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    tmp = tempfile.mkdtemp(prefix="sfm_kst_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        cmd = [prof, "--kernel-trace", "--stats", "--output-format", "csv", "-d", tmp, "-o", "k", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child",
               "--n-cam", str(args.n_cam), "--n-pt", str(args.n_pt), "--match-frames", str(args.match_frames)]
        try:
            r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=240)
        except subprocess.TimeoutExpired:
            log("kernel-stats pass timed out")
            return None
        files = glob.glob(os.path.join(tmp, "**", "*kernel_stats.csv"), recursive=True)
        if r.returncode != 0 or not files:
            log(f"kernel-stats pass failed (rc {r.returncode}): {r.stderr[-400:]}")
            return None
        for row in csv.DictReader(open(files[0])):
            name = row.get("Name", "")
            if kernel_prefix in name:
                return {"mean_ms": float(row["AverageNs"]) * 1e-6, "launches": int(row["Calls"]), "kernel": name}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return None


def pmc_measure(args, kernel_regex="schur_kernel", child="--pmc-child"):
    """HBM bytes and MFMA-busy cycles per launch of the Schur kernel (or the
    matcher: child --pmc-child-match), measured now by rocprofv3 --pmc passes
    over a child run of the same configuration.
    Returns None when rocprofv3 is unavailable or a pass fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    vals = {}
    tmp = tempfile.mkdtemp(prefix="sfm_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        for k, counters in enumerate(PMC_PASSES):
            d = os.path.join(tmp, f"pass{k}")
            cmd = [prof, "--pmc", *counters, "--kernel-include-regex", kernel_regex, "--output-format", "csv",
                   "-d", d, "-o", "p", "--", sys.executable, os.path.abspath(__file__), child,
                   "--n-cam", str(args.n_cam), "--n-pt", str(args.n_pt), "--match-frames", str(args.match_frames)]
            try:
                r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=240)
            except subprocess.TimeoutExpired:
                log(f"pmc pass {counters} timed out")
                return None
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                log(f"pmc pass {counters} failed (rc {r.returncode}): {r.stderr[-400:]}")
                return None
            for row in csv.DictReader(open(files[0])):
                name = row.get("Kernel_Name", "")
                if ", true>" in name:   # the solve's first pass also forms the point scales
                    continue
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if "FETCH_SIZE" not in vals or "WRITE_SIZE" not in vals:
        return None
    mean = {c: sum(v) / len(v) for c, v in vals.items()}
    out = {"fetch_bytes": 2.0 * 1024.0 * mean["FETCH_SIZE"],   # gfx950: FETCH_SIZE counts half (guide §HBM)
           "write_bytes": 1024.0 * mean["WRITE_SIZE"], "launches": len(vals["FETCH_SIZE"])}
    out["traffic"] = out["fetch_bytes"] + out["write_bytes"]
    for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
        if c in mean:
            out[c] = mean[c]
    return out


def bench_loop(ctx, n_img, cpu=True, cpu_images=16, fixed_writeback=False, imgs=None):
    """C5: SequentialActuator over the synthetic closed orbit (src/main.cpp:99-108):
    init + BA, then addSingleImage + BA per image, a fresh BundleAdjuster per
    call.  Images are generated before the timed region (they stand for what
    detectAndCompute leaves behind); the timed region is the whole loop.
    fixed_writeback: the write-back without the Image::setIntrinsic quirk, so
    the world keeps growing to the end of the orbit."""
    seq = api.OrbitSequence(n_img=n_img)
    if imgs is None:
        t0 = time.time()
        imgs = [seq.image(k) for k in range(n_img)]
        log(f"loop: {n_img} images generated in {time.time() - t0:.1f}s "
            f"({np.mean([len(i['kp']) for i in imgs]):.0f} keypoints each)")
    so = api.seq_default_options()
    so.fixed_writeback = 1 if fixed_writeback else 0
    lp = api.SeqLoop(ctx, so)
    steps = []
    t0 = time.perf_counter()
    lp.init(imgs[0], imgs[1])
    lp.bundle_adjust()
    steps.append(lp.step())
    for k in range(2, n_img):
        lp.add(imgs[k])
        lp.bundle_adjust()
        steps.append(lp.step())
    ctx.synchronize()
    dt = time.perf_counter() - t0
    lp.close()
    stage = {f: sum(getattr(s, "seconds_" + f) for s in steps)
             for f in ("local_match", "global_match", "geometry", "ba")}
    iters = sum(s.ba.iterations for s in steps)
    last = steps[-1]
    out = {"metric": "C5 incremental loop images/sec" + (", fixed write-back" if fixed_writeback else ""),
           "value": n_img / dt, "unit": "images/s",
           "seconds": dt, "stage_seconds": stage,
           "ba_calls": len(steps), "ba_lm_iterations": iters,
           "ba_lm_iters_per_sec_in_loop": iters / max(stage["ba"], 1e-12),
           "kept_images": 1 + sum(s.kept for s in steps),
           "world_points": last.world_points, "world_observations": last.world_observations,
           "final_ba": {"rmse_initial": last.ba.rmse_initial, "rmse_final": last.ba.rmse_final,
                        "iterations": last.ba.iterations, "observations": last.ba_observations},
           # the world stops growing once PnP fails on the images after the
           # setIntrinsic quirk has rewritten the shared camera; every later
           # call re-adjusts a world the previous write-back perturbed, so
           # its RMSE is not a measure of the solver
           "last_growth_ba": next(({"image": k + 1, "rmse_initial": s.ba.rmse_initial,
                                    "rmse_final": s.ba.rmse_final, "iterations": s.ba.iterations,
                                    "observations": s.ba_observations}
                                   for k, s in reversed(list(enumerate(steps)))
                                   if s.world_points > (steps[k - 1].world_points if k else 0)), None),
           "config": {"workload": f"C5 SequentialActuator loop, {n_img}-image synthetic closed orbit "
                                  f"({seq.cfg.n_landmarks} landmarks, tracks ~{seq.cfg.track_mean:g} images, "
                                  f"{seq.cfg.n_clutter} clutter keypoints/image), LocalFrame + GlobalFrame "
                                  "mutual matching and a fresh BundleAdjuster per image, "
                                  + ("fixed write-back (Image::setIntrinsic quirk off)" if fixed_writeback else
                                     "Image::setIntrinsic quirk on (reference write-back)"),
                       "host_malloc": "SFM_CTX_TUNE_HOST_MALLOC (opt-in, bench process only)"}}
    out["images"] = imgs
    log(f"loop{' (fixed write-back)' if fixed_writeback else ''}: {n_img} images in {dt:.2f}s "
        f"({n_img / dt:.1f} images/s), kept {out['kept_images']}, stages "
        + ", ".join(f"{k} {v:.2f}s" for k, v in stage.items())
        + f"; {iters} LM iterations; world {last.world_points} pts / {last.world_observations} obs")
    if cpu:
        try:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import _helpers as H   # oracle loader (test infrastructure: the CPU baseline only)
            model, nth = host_cpu()
            n = min(cpu_images, n_img)
            ol = H.OracleSeqLoop(threads=nth)
            t1 = time.perf_counter()
            ol.init(imgs[0], imgs[1])
            ol.bundle_adjust()
            for k in range(2, n):
                ol.add(imgs[k])
                ol.bundle_adjust()
            cdt = time.perf_counter() - t1
            ol.close()
            gpu_first = sum(s.seconds_local_match + s.seconds_global_match + s.seconds_geometry + s.seconds_ba
                            for s in steps[:n - 1])
            out["cpu_baseline"] = {"value": n / cdt, "unit": "images/s", "cores": nth, "kind": "port",
                                   "cpu_model": model,
                                   "sample": f"the first {n} images of the same sequence through the loop oracle "
                                             f"(CPU matcher + Ceres-semantics solver, {nth} threads), "
                                             f"{cdt:.1f} s wall; the GPU loop spent {gpu_first:.2f} s on "
                                             "those images"}
            log(f"cpu baseline loop: {n} images in {cdt:.1f}s")
        except Exception as ex:
            log(f"cpu baseline loop unavailable: {ex}")
    return out


def synth_fpairs(n_pairs, n_match, outlier_frac=0.3, seed=0xF3, w=1920, h=1080, f=1400.0):
    """Synthetic putative matches for the geometric filter: per pair, n_match
    projections of random points into two views (0.5 px noise), a fraction
    replaced by uniform clutter in the second view."""
    rng = np.random.default_rng(seed)
    K = np.array([[f, 0, w / 2], [0, f, h / 2], [0, 0, 1.0]])
    xs = []
    for _ in range(n_pairs):
        wv = rng.normal(0, 0.15, 3)
        th = np.linalg.norm(wv)
        k = wv / th
        Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        R = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
        t = np.array([-0.6, rng.normal(0, 0.1), rng.normal(0, 0.1)])
        X = np.stack([rng.uniform(-3, 3, n_match), rng.uniform(-2, 2, n_match), rng.uniform(5, 12, n_match)], 1)
        p1 = (K @ X.T).T
        p2 = (K @ (R @ X.T + t[:, None])).T
        u1 = p1[:, :2] / p1[:, 2:] + rng.normal(0, 0.5, (n_match, 2))
        u2 = p2[:, :2] / p2[:, 2:] + rng.normal(0, 0.5, (n_match, 2))
        out = rng.random(n_match) < outlier_frac
        u2[out] = np.stack([rng.uniform(0, w, out.sum()), rng.uniform(0, h, out.sum())], 1)
        xs.append(np.concatenate([u1, u2], 1))
    return xs, [(w, h, w, h)] * n_pairs


def bench_radial3_percam(ctx, n_cam=200, n_pt=50_000, k=10, steps=2):
    """reconstruction()'s one intrinsics group per camera
    (sparseBuilder.cpp:1292-1299) under OpenMVG's PINHOLE_CAMERA_RADIAL3: the
    arrow is as wide as the band (6 n_cam intrinsics columns), so the RCS is
    dense, and a point's 2 x 6k F rows exceed a chunk tile, so every point
    takes the general path.  C2-sized (the per-camera arrow multiplies the
    RCS by 2 and the product terms by ~4 against pinhole)."""
    t0 = time.time()
    sc = c4_scene(n_cam, n_pt, k=k, seed=0x5F3D0024, vis=0, model=abi.SFM_CAM_RADIAL3, n_intr=n_cam)
    plan = api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
    t_plan = time.time() - t0
    info = plan.info()
    plan.run()   # warm-up
    ctx.synchronize()
    t1 = time.perf_counter()
    iters = 0
    for _ in range(steps):
        rc, summ = plan.run()
        iters += summ.iterations
    ctx.synchronize()
    dt = time.perf_counter() - t1
    plan.close()
    shape = api.ba_describe(sc["problem"])
    out = {"metric": "BA LM-iters/sec, RADIAL3 with one intrinsics block per camera", "value": iters / dt,
           "unit": "LM-iters/s", "ms_per_iteration": dt / max(iters, 1) * 1e3,
           "lm_iterations_per_solve": summ.iterations, "rmse_initial": summ.rmse_initial,
           "rmse_final": summ.rmse_final, "rcs_dim": info.rcs_dim, "dense": bool(shape.dense),
           "general_points": shape.n_general_pts, "product_terms": shape.n_pterms, "host_plan_seconds": t_plan,
           "config": {"workload": f"{n_cam} cams / {n_pt} pts / {sc['n_obs']} obs, banded k={k}, "
                                  "Pinhole_Intrinsic_Radial_K3 per camera (reconstruction()'s grouping), HuberLoss(4)"}}
    log(f"BA radial3 per-camera: {iters} LM iterations in {dt:.3f}s -> {iters / dt:.1f} it/s, rcs {info.rcs_dim}, "
        f"dense {bool(shape.dense)}, {shape.n_general_pts} general points, plan {t_plan:.1f}s, "
        f"rmse {summ.rmse_initial:.4f}->{summ.rmse_final:.4f}")
    return out


def bench_dense_s(ctx, n_cam=1000, n_pt=500_000, k=10, steps=2, model=0):
    """SURVEY §8(d)'s dense-S stress case: random-k visibility (vis_mode 1),
    so every camera pair can share points, the reduced camera system is dense
    (nF = 6 (n_cam - 1) + 4) and the general-point path plus the blocked dense
    Cholesky (ba_bcr.hip dense_*) carry the solve.  C4's sizes.
    model = SFM_CAM_RADIAL3: C4's banded geometry under OpenMVG's
    PINHOLE_CAMERA_RADIAL3 residual: the chunk path with
    6-row intrinsics slots and the BCR band solver, as pinhole."""
    t0 = time.time()
    r3 = model == abi.SFM_CAM_RADIAL3
    sc = c4_scene(n_cam, n_pt, k=k, seed=0x5F3D0004 if r3 else 0x5F3D0014, vis=0 if r3 else 1, model=model)
    plan = api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
    t_plan = time.time() - t0
    info = plan.info()
    plan.run()   # warm-up
    ctx.synchronize()
    t1 = time.perf_counter()
    iters = 0
    for _ in range(steps):
        rc, summ = plan.run()
        iters += summ.iterations
    ctx.synchronize()
    dt = time.perf_counter() - t1
    plan.close()
    nF = info.rcs_dim
    dense = bool(api.ba_describe(sc["problem"]).dense)
    out = {"metric": "BA LM-iters/sec, PINHOLE_CAMERA_RADIAL3 residual model" if r3 else
                     "BA LM-iters/sec, dense reduced camera system (random-k visibility)",
           "value": iters / dt, "unit": "LM-iters/s", "ms_per_iteration": dt / max(iters, 1) * 1e3,
           "lm_iterations_per_solve": summ.iterations, "rmse_initial": summ.rmse_initial,
           "rmse_final": summ.rmse_final, "rcs_dim": nF, "dense": dense,
           "rcs_factor_flops_per_iteration": nF ** 3 / 3.0 if dense else None, "host_plan_seconds": t_plan,
           "config": {"workload": f"{n_cam} cams / {n_pt} pts / {sc['n_obs']} obs, random k={k} visibility "
                                  "(SURVEY §8(d) dense-S stress variant of C4), HuberLoss(4)"}}
    if r3:
        out["config"] = {"workload": f"C4 geometry ({n_cam} cams / {n_pt} pts / {sc['n_obs']} obs, banded k={k}), "
                                     "OpenMVG Pinhole_Intrinsic_Radial_K3 residual {f, ppx, ppy, k1, k2, k3} "
                                     "(one shared block, ADJUST_ALL), HuberLoss(4); chunk path + BCR band solver"}
    log(f"BA {'radial3' if r3 else 'dense-S'}: {iters} LM iterations in {dt:.3f}s -> {iters / dt:.1f} it/s, rcs {nF}, plan {t_plan:.1f}s, "
        f"rmse {summ.rmse_initial:.4f}->{summ.rmse_final:.4f}")
    return out


def bench_filter(ctx, n_pairs, n_match, cpu=True, cpu_pairs=32):
    """sparseBuilder::filter()'s GeometricFilter_FMatrix_AC(4.0, 2048) over a
    synthetic collection of putative pairs."""
    xs, whs = synth_fpairs(n_pairs, n_match)
    api.fmatrix_ac(ctx, xs[:8], whs[:8])   # warm-up (code object, caches)
    ctx.synchronize()
    t0 = time.perf_counter()
    res = api.fmatrix_ac(ctx, xs, whs)
    dt = time.perf_counter() - t0
    kms = C.c_double(0.0)
    abi.load().sfm_ctx_last_kernel_ms(ctx.h, C.byref(kms))
    iters = sum(r["iterations"] for r in res)
    kept = sum(r["n_inliers"] > 0 for r in res)
    out = {"metric": "geometric filter pairs/sec (F-matrix AC-RANSAC, 2048 iterations)", "value": n_pairs / dt,
           "unit": "pairs/s", "seconds": dt, "pairs": n_pairs, "matches_per_pair": n_match,
           "ransac_iterations_per_sec": iters / dt, "pairs_kept": kept,
           # the timed call includes the host normalisation, the uploads and
           # the result download; the kernel alone (HIP events):
           "kernel_ms": kms.value if kms.value > 0 else None,
           "kernel_pairs_per_sec": n_pairs / (kms.value * 1e-3) if kms.value > 0 else None,
           "inliers": int(sum(r["n_inliers"] for r in res)),
           "workload": f"{n_pairs} pairs x {n_match} putative matches (30% clutter), 1920x1080 views, "
                       "GeometricFilter_FMatrix_AC(4.0, 2048) semantics (sparseBuilder.cpp:1179-1186); "
                       "time includes upload, normalisation and download"}
    log(f"filter: {n_pairs} pairs in {dt:.3f}s -> {n_pairs / dt:.0f} pairs/s ({iters / dt:.3g} RANSAC it/s), "
        f"{kept} kept")
    if cpu:
        try:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import _helpers as H   # oracle loader (test infrastructure: the CPU baseline only)
            lib = H.oracle()
            lib.orc_fmatrix_ac.restype = C.c_int
            lib.orc_fmatrix_ac.argtypes = [C.c_int64, abi.i64p, abi.f64p, abi.i32p, C.POINTER(abi.FMatrixOpts),
                                           C.POINTER(abi.FMatrixResult), abi.i32p, C.c_int32]
            model, nth = host_cpu()
            n = min(cpu_pairs, n_pairs)
            off, xy, wh = api._fmatrix_inputs(xs[:n], whs[:n])
            r = (abi.FMatrixResult * n)()
            inl = np.zeros(int(off[-1]), np.int32)
            t1 = time.perf_counter()
            lib.orc_fmatrix_ac(n, abi.ptr(off, abi.i64p), abi.ptr(xy, abi.f64p), abi.ptr(wh, abi.i32p),
                               C.byref(api.fmatrix_opts()), r, abi.ptr(inl, abi.i32p), nth)
            cdt = time.perf_counter() - t1
            out["cpu_baseline"] = {"value": n / cdt, "unit": "pairs/s", "cores": nth, "kind": "port",
                                   "cpu_model": model,
                                   "sample": f"the first {n} pairs of the same collection through the filter "
                                             f"oracle (OpenMP over pairs, {nth} threads), {cdt:.1f} s wall"}
            log(f"cpu baseline filter: {n} pairs in {cdt:.1f}s")
        except Exception as ex:
            log(f"cpu baseline filter unavailable: {ex}")
    return out


def loop_replica_line(r, seconds, images):
    """The C5 line at N > 1: N independent replicas of the same sequence, one
    per GPU (the loop does not shard).  `r` is rank 0's
    bench_loop result, `seconds` every rank's loop wall time in rank order.
    `value` is the aggregate images/s over the slowest replica (weak scaling:
    N sequences, not one sequence N times faster); the metric name says so and
    each replica's own rate is reported beside it, so the aggregate is not
    read as a speedup of one reconstruction."""
    world, t_max = len(seconds), max(seconds)
    out = dict(r)
    out.update(metric=f"C5 incremental loop images/sec, fixed write-back, aggregate of {world} independent "
                      f"replicas (one sequence per GPU)",
               value=world * images / t_max, seconds=t_max, replicas=world,
               per_replica_images_per_sec=[images / t for t in seconds],
               slowest_replica_images_per_sec=images / t_max,
               scaling="weak (independent sequences, one per GPU; not a speedup of one sequence; DESIGN.md §7)")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # C4 solves are ~5 ms each: 20 timed after 3 warm-up solves keep the timed
    # region (~0.1 s) clear of clock ramp-up and host jitter (5 after 1 read
    # 2-3 % low box to box); only the BA sections use these counts
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-pt", type=int, default=500_000)
    ap.add_argument("--n-cam", type=int, default=1000)
    ap.add_argument("--match-frames", type=int, default=500)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-match", action="store_true")
    ap.add_argument("--no-snavely", action="store_true")
    ap.add_argument("--no-radial3", action="store_true")
    ap.add_argument("--no-loop", action="store_true")
    ap.add_argument("--loop-images", type=int, default=300)
    ap.add_argument("--no-filter", action="store_true")
    ap.add_argument("--no-dense", action="store_true")
    ap.add_argument("--filter-pairs", type=int, default=2000)
    ap.add_argument("--filter-matches", type=int, default=1000)
    # diagnostic: rank 0's shard of an N-way landmark partition on this one GPU,
    # with a no-op all-reduce (per-rank kernel times of the N-GPU run; the
    # solve itself is then not the global one, so the result is not a bench line)
    ap.add_argument("--fake-world", type=int, default=0)
    # N > 1 without an RCCL communicator: the host-staged gloo all-reduce only
    # when asked for (the number is then labelled in config.transport)
    ap.add_argument("--allow-host-allreduce", action="store_true")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-child-match", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.pmc_child:
        pmc_child(args)
        return
    if args.pmc_child_match:
        pmc_child_match(args)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("SFM_BENCH_LAUNCH_CHECK"):   # CPU test of the self-launch: no GPU work
        # one write of the whole line (< PIPE_BUF): the ranks share the pipe
        os.write(1, (json.dumps({"rank": rank, "world": world, "local_rank": local_rank, "gpus": args.gpus})
                     + "\n").encode())
        return
    if os.environ.get("SFM_BENCH_SAME_DEVICE"):   # rehearsal of N>1 on a one-GPU box
        local_rank = 0
    if args.gpus != world:
        # the launcher's WORLD_SIZE is the truth; a mismatch is reported, never hidden
        log(f"WARNING: --gpus {args.gpus} but WORLD_SIZE {world}; running and reporting {world} rank(s)")
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    import torch
    if torch.cuda.is_available():   # torch's synchronize() below targets this rank's GPU, not GPU 0
        torch.cuda.set_device(local_rank)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize() if torch.cuda.is_available() else None

    def max_over_ranks(v):
        if dist is None:
            return v
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_over_ranks(v):   # every rank's value, in rank order
        if dist is None:
            return [v]
        got = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(got, torch.tensor([v], dtype=torch.float64))
        return [float(t.item()) for t in got]

    comm_id = None
    transport = "none"
    if world > 1:
        obj = [None]
        if rank == 0:
            try:
                obj = [api.comm_unique_id()]
            except Exception as ex:  # no RCCL: every rank falls back together
                log(f"RCCL unique id unavailable ({ex})")
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]
    ctx = None
    if comm_id is not None:
        try:
            ctx = api.Context(device=local_rank, rank=rank, world_size=world, comm_id=comm_id,
                              flags=abi.SFM_CTX_TIME_KERNELS)
            transport = "rccl"
        except Exception as ex:
            log(f"RCCL communicator failed ({ex})")
    if world > 1:   # every rank must agree on the transport
        ok = torch.tensor([1 if ctx is not None else 0])
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            if ctx is not None:
                ctx.close()
            if not args.allow_host_allreduce:
                raise RuntimeError("RCCL communicator unavailable on some rank; refusing to benchmark over the "
                                   "host gloo all-reduce (pass --allow-host-allreduce to measure that transport)")

            def host_allreduce(a, op):
                dist.all_reduce(torch.from_numpy(a), op=dist.ReduceOp.MAX if op == 1 else dist.ReduceOp.SUM)

            ctx = api.Context(device=local_rank, rank=rank, world_size=world, allreduce=host_allreduce,
                              flags=abi.SFM_CTX_TIME_KERNELS)
            transport = "gloo-host (RCCL unavailable)"
            log("falling back to the host-staged gloo all-reduce")
    elif args.fake_world > 1:
        ctx = api.Context(device=local_rank, rank=0, world_size=args.fake_world,
                          flags=abi.SFM_CTX_DIAG_NO_EXCHANGE | abi.SFM_CTX_TIME_KERNELS)
        transport = f"none (diagnostic: shard 0 of {args.fake_world}, exchanges skipped on the device)"
    else:
        # opt-in host malloc setting for this short-lived process
        ctx = api.Context(device=local_rank, flags=abi.SFM_CTX_TUNE_HOST_MALLOC | abi.SFM_CTX_TIME_KERNELS)

    # the committed PMC summary was measured on the default C4/C3 sizes at N=1
    pmc_ok = (world == 1 and args.n_pt == 500_000 and args.n_cam == 1000 and args.match_frames == 500)

    # ---------------- BA (C4) ----------------
    t0 = time.time()
    sc = c4_scene(args.n_cam, args.n_pt)
    log(f"scene: {sc['n_obs']} obs in {time.time() - t0:.1f}s")
    t0 = time.time()
    plan = api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
    info = plan.info()
    log(f"plan: {time.time() - t0:.1f}s chunks={info.n_chunks} D={info.band_blocks} "
        f"rcs={info.rcs_dim} shard_obs={info.shard_obs}")
    for _ in range(args.warmup):
        plan.run()
    ctx.synchronize()
    barrier()
    t0 = time.perf_counter()
    iters = 0
    summ = None
    for _ in range(args.steps):
        rc, summ = plan.run()
        iters += summ.iterations
    ctx.synchronize()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    value = iters / dt
    obs_per_sec = iters * sc["n_obs"] / dt
    # the roofline's launch time: every Schur launch but each solve's first
    # (which also forms the point scales), over separate solves after the timed
    # region (the timed solves carry no events: an event pair serialises the
    # stream for ~12 us)
    os.environ["SFM_SCHUR_TIME_ALL"] = "1"
    schur_ms, schur_n = 0.0, 0
    for _ in range(max(3, min(args.steps, 10))):
        plan.run()
        inf = plan.info()
        schur_ms += inf.schur_ms_total
        schur_n += inf.schur_launches
    ctx.synchronize()
    del os.environ["SFM_SCHUR_TIME_ALL"]
    schur_avg_ms = schur_ms / max(schur_n, 1)
    flops = info.schur_flops_per_iter
    achieved = flops / (schur_avg_ms * 1e-3) / 1e12 if schur_n else 0.0
    # (iterations per solve printed: a --fake-world shard solves its own
    # problem, whose accept / reject mix differs from the whole scene's)
    log(f"BA: {iters} LM iterations in {dt:.3f}s -> {value:.1f} it/s ({summ.iterations} per solve), rmse "
        f"{summ.rmse_initial:.4f}->{summ.rmse_final:.4f}, schur avg {schur_avg_ms:.3f} ms")
    fake_est = None
    if args.fake_world > 1:
        # --fake-world skips every exchange on the device, so its rate leaves
        # out the per-iteration RCS all-reduce and scalar all-gather.  Estimate
        # them as SURVEY §8(e) does: a ring all-reduce of the RCS over one
        # 153 GB/s xGMI link, 2 (W-1)/W bytes, plus an assumed 10 us latency
        # per collective (two per iteration).  An estimate, not a measurement.
        W = args.fake_world
        iw = ctx.lib.sfm_ba_intr_width(0)
        ncam, nintr, D = info.n_cam_active, info.n_intr_active, info.band_blocks
        nF = 6 * ncam + iw * nintr
        rcs_doubles = ncam * (D + 1) * 36 + nintr * ncam * 6 * iw + (nintr * iw) ** 2 + 3 * nF + 1
        ex_us = 2 * (W - 1) / W * rcs_doubles * 8 / 153e9 * 1e6 + 2 * 10.0
        it_us = dt / iters * 1e6
        fake_est = {"rank0_us_per_iter": it_us, "exchange_us_per_iter_est": ex_us,
                    "rcs_bytes": rcs_doubles * 8,
                    "lm_iters_per_s_with_exchange_est": 1e6 / (it_us + ex_us),
                    "model": "ring all-reduce over one 153 GB/s xGMI link + 2 x 10 us collective latency"}
        log(f"fake-world {W}: rank 0 {it_us:.1f} us/iter without exchanges; estimated exchange "
            f"{ex_us:.1f} us/iter (RCS {rcs_doubles * 8 / 1e6:.2f} MB) -> "
            f"~{fake_est['lm_iters_per_s_with_exchange_est']:.0f} LM-iters/s with exchanges (estimate)")

    # PCIe-inclusive: one sfm_ba_solve from host buffers (upload, symbolic
    # plan, solve, download) -- reported beside the bench value, never as it
    pcie = None
    if world == 1:
        def host_solve():
            e_h, i_h, x_h = sc["extr"].copy(), sc["intr"].copy(), sc["X"].copy()
            t1 = time.perf_counter()
            rc_h, s_h = api.ba_solve(ctx, sc["problem"], e_h, i_h, x_h)
            return s_h, time.perf_counter() - t1
        s_c, dt_c = host_solve()     # plan built from the host buffers (kept in the context)
        s_w, dt_w = host_solve()     # same structure again: plan reused, values re-uploaded
        pcie = {"value": s_w.iterations / dt_w, "unit": "LM-iters/s", "seconds": dt_w,
                "iterations": s_w.iterations,
                "what": "sfm_ba_solve from host buffers with the context's cached plan (same problem "
                        "structure as the previous call): value upload + device gather + LM solve + download",
                "cold": {"value": s_c.iterations / dt_c, "seconds": dt_c,
                         "what": "first sfm_ba_solve: upload + symbolic plan + LM solve + download"}}
        log(f"BA from host buffers: cold {dt_c * 1e3:.1f} ms, plan reused {dt_w * 1e3:.1f} ms "
            f"for {s_w.iterations} iterations")
        abi.load().sfm_ba_cache_clear(ctx.h)

    # ---------------- BA, BAL residual model ----------------
    snav = None
    if not args.no_snavely:
        ssc = c4_scene(args.n_cam, args.n_pt, model=abi.SFM_CAM_SNAVELY)
        splan = api.BAPlan(ctx, ssc["problem"], ssc["extr"], ssc["intr"], ssc["X"])
        for _ in range(args.warmup):
            splan.run()
        ctx.synchronize()
        barrier()
        t0 = time.perf_counter()
        s_iters = 0
        for _ in range(args.steps):
            rc, ssum = splan.run()
            s_iters += ssum.iterations
        ctx.synchronize()
        barrier()
        sdt = max_over_ranks(time.perf_counter() - t0)
        # the Schur launch time over separate solves (as for C4 above)
        os.environ["SFM_SCHUR_TIME_ALL"] = "1"
        s_ms, s_n = 0.0, 0
        for _ in range(3):
            splan.run()
            inf = splan.info()
            s_ms += inf.schur_ms_total
            s_n += inf.schur_launches
        ctx.synchronize()
        del os.environ["SFM_SCHUR_TIME_ALL"]
        s_avg = s_ms / max(s_n, 1)
        s_flops = splan.info().schur_flops_per_iter
        s_ach = s_flops / (s_avg * 1e-3) / 1e12 if s_n else 0.0
        snav = {"metric": "BA LM-iters/sec, SnavelyReprojectionError (BAL) residual model",
                "value": s_iters / sdt, "unit": "LM-iters/s", "ms_per_step": sdt / args.steps * 1e3,
                "obs_per_sec": s_iters * ssc["n_obs"] / sdt, "lm_iterations_per_solve": ssum.iterations,
                "rmse_initial": ssum.rmse_initial, "rmse_final": ssum.rmse_final,
                "config": {"workload": f"C4 geometry ({args.n_cam} cams / {args.n_pt} pts / "
                                       f"{ssc['n_obs']} obs), SnavelyReprojectionError.h model "
                                       "(f, l1, l2 per camera block; one shared block), HuberLoss(4)"},
                "roofline": {"bound": "mfma", "achieved": s_ach, "peak": FP64_PEAK_TF, "unit": "TFLOP/s",
                             "frac": s_ach / FP64_PEAK_TF, "kernel": "schur_kernel<SNAVELY>",
                             "per_launch_ms": s_avg}}
        log(f"BA snavely: {s_iters} LM iterations in {sdt:.3f}s -> {s_iters / sdt:.1f} it/s, rmse "
            f"{ssum.rmse_initial:.4f}->{ssum.rmse_final:.4f}")
        splan.close()
        del ssc

    # ---------------- matching (C3) ----------------
    match = None
    if not args.no_match:
        nf, nkp = args.match_frames, 4096
        desc = api.synth_descriptors(nf, nkp)
        off = np.arange(nf + 1, dtype=np.int64) * nkp
        pairs = api.exhaustive_pairs(nf)
        lo = len(pairs) * rank // world
        hi = len(pairs) * (rank + 1) // world
        mplan = api.MatchPlan(ctx, desc, off)
        mplan.run(pairs[lo:min(hi, lo + 512)], count=False)  # warm-up
        ctx.synchronize()
        barrier()
        t1 = time.perf_counter()
        mplan.run(pairs[lo:hi], count=False)
        ctx.synchronize()
        barrier()
        mdt = max_over_ranks(time.perf_counter() - t1)
        kms, kl = mplan.last_ms()
        tops = (hi - lo) * 2.0 * 128 * nkp * nkp / (kms * 1e-3) / 1e12
        match = {"metric": "SIFT match pairs/sec", "value": len(pairs) / mdt, "unit": "pairs/s",
                 "config": {"workload": f"C3 all-pairs ratio-0.8 matching, {nf} frames x {nkp} x "
                                        "128-D uint8 (RootSIFT-like synthetic), "
                                        f"{len(pairs)} exhaustive pairs"},
                 "dtype": "u8 (i8 MFMA, i32 accumulate: exact)",
                 "roofline": {"bound": "mfma", "achieved": tops, "peak": I8_PEAK_TOPS,
                              "unit": "TOP/s", "frac": tops / I8_PEAK_TOPS,
                              "traffic": pmc_traffic("match_top2_kernel", largest=True) if pmc_ok else None,
                              "kernel": "match_top2_kernel",
                              "per_launch_ms": kms / max(kl, 1)},
                 "digest": mplan.digest()}
        log(f"match: {len(pairs)} pairs in {mdt:.3f}s -> {len(pairs) / mdt:.0f} pairs/s, "
            f"{tops:.0f} TOP/s")
        # the legacy exact matcher (LocalFrame/GlobalFrame crossCheck):
        # MUTUAL mode on the first tenth of the pair list (two top-1 passes per pair)
        msub = pairs[: max(1, len(pairs) // 10)]
        mlo, mhi = len(msub) * rank // world, len(msub) * (rank + 1) // world
        ctx.synchronize()
        barrier()
        t1 = time.perf_counter()
        mplan.run(msub[mlo:mhi], mode=abi.SFM_MATCH_MUTUAL, count=False)
        ctx.synchronize()
        barrier()
        udt = max_over_ranks(time.perf_counter() - t1)
        match["mutual"] = {"metric": "SIFT mutual (crossCheck) match pairs/sec", "value": len(msub) / udt,
                           "unit": "pairs/s", "pairs": len(msub),
                           "workload": "first 10% of the C3 pair list, BFMatcher(NORM_L2, crossCheck) "
                                       "semantics (LocalFrame.h:31-47), exact"}
        log(f"match mutual: {len(msub)} pairs in {udt:.3f}s -> {len(msub) / udt:.0f} pairs/s")
        # the reference's live default, "AUTO" -> cascade hashing (SURVEY §8(f)
        # row 1): index (zero-mean, codes, buckets of every image of the list;
        # replicated per rank) + this rank's part of the pair list, timed together
        mplan.run(pairs[:64], mode=abi.SFM_MATCH_CASCADE, count=False)   # warm-up
        ctx.synchronize()
        barrier()
        t1 = time.perf_counter()
        mplan.cascade_index(pairs)
        ctx.synchronize()
        t_idx = time.perf_counter() - t1
        mplan.run(pairs[lo:hi], mode=abi.SFM_MATCH_CASCADE, count=False)
        ctx.synchronize()
        barrier()
        cdt = max_over_ranks(time.perf_counter() - t1)
        ckms, ckl = mplan.last_ms()
        # algorithmic bytes per pair: both images' hashed tables read once
        # (database I: descriptors, codes, 6 bucket lists, bucket offsets;
        # queries J: descriptors, codes, bucket ids) + the per-query result
        bpp = nkp * (128 + 16 + 6 * 4) + 6 * 1025 * 4 + nkp * (128 + 16 + 16) + nkp * 8
        cgbs = (hi - lo) * bpp / (ckms * 1e-3) / 1e9
        match["cascade"] = {
            "metric": "SIFT cascade-hashing match pairs/sec", "value": len(pairs) / cdt,
            "unit": "pairs/s", "pairs": len(pairs), "index_ms": t_idx * 1e3,
            "workload": "C3 pair list, Cascade_Hashing_Matcher_Regions(0.8) semantics "
                        "(sparseBuilder.cpp:911-914, the reference's AUTO default); "
                        "time includes hashing every image",
            # not an HBM roofline: the kernel is bound by dependent bucket
            # gathers (L2 / LDS latency); the per-pair table bytes
            # below exceed what the counters see reaching HBM (the tables of an
            # image are re-read from L2 by every pair that uses it)
            "roofline": {"bound": "gathers", "achieved": cgbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": cgbs / HBM_PEAK_GBS,
                         "traffic": pmc_traffic("casc_match_lds_kernel", largest=True) if pmc_ok else None,
                         "kernel": "casc_match_lds_kernel", "per_launch_ms": ckms / max(ckl, 1),
                         "algorithmic_bytes_per_pair": bpp,
                         "note": "bound = dependent gathers, not HBM: traffic <= algorithmic bytes (tables "
                                 "reused from L2 across pairs); frac is table bytes touched / HBM peak, "
                                 "not a bandwidth utilisation"},
            "digest": mplan.digest()}
        log(f"match cascade: {len(pairs)} pairs in {cdt:.3f}s (index {t_idx * 1e3:.1f} ms) -> "
            f"{len(pairs) / cdt:.0f} pairs/s, match kernels {ckms:.1f} ms")

    # ---------------- incremental loop (C5) ----------------
    loop = loop_fixed = None
    if world == 1 and rank == 0 and not args.no_loop and args.fake_world <= 1:
        loop = bench_loop(ctx, args.loop_images, cpu=not args.no_cpu_baseline)
        loop_fixed = bench_loop(ctx, args.loop_images, cpu=False, fixed_writeback=True, imgs=loop.pop("images"))
        loop_fixed.pop("images", None)
    elif world > 1 and not args.no_loop:
        # C5 at N > 1: replicas only (DESIGN.md §7 -- the loop is host bound,
        # one image after another).  Every rank runs its own sequence on a
        # one-rank context of its GPU; rank 0 reports the aggregate and every
        # replica's own rate (loop_replica_line).
        lctx = api.Context(device=local_rank)
        barrier()
        r = bench_loop(lctx, args.loop_images, cpu=False, fixed_writeback=True)
        r.pop("images", None)
        lctx.synchronize()
        lctx.close()
        secs = all_over_ranks(r["seconds"])
        if rank == 0:
            loop_fixed = loop_replica_line(r, secs, args.loop_images)
            log(f"loop replicas: {world} x {args.loop_images} images, slowest rank {max(secs):.2f}s "
                f"-> {loop_fixed['value']:.1f} images/s aggregate")

    # ---------------- dense-S stress case ----------------
    dense_s = None
    if world == 1 and rank == 0 and not args.no_dense and args.fake_world <= 1:
        dense_s = bench_dense_s(ctx)
    radial3 = radial3_percam = None
    if world == 1 and rank == 0 and not args.no_radial3 and args.fake_world <= 1:
        radial3 = bench_dense_s(ctx, model=abi.SFM_CAM_RADIAL3)
        radial3_percam = bench_radial3_percam(ctx)

    # ---------------- geometric filter ----------------
    filt = None
    if world == 1 and rank == 0 and not args.no_filter and args.fake_world <= 1:
        filt = bench_filter(ctx, args.filter_pairs, args.filter_matches, cpu=not args.no_cpu_baseline)

    cpu = None
    cpu_match = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline_ba(sc)
            log(f"cpu baseline BA: {cpu['value']:.4f} it/s on {cpu['cores']} threads, "
                f"{cpu['single_thread']['value']:.4f} it/s on 1")
            if match is not None:
                cpu_match = cpu_baseline_match(desc, 4096, pairs)
                match["cpu_baseline"] = cpu_match
                match["cascade"]["cpu_baseline"] = cpu_baseline_cascade(desc, 4096)
                log(f"cpu baseline cascade: {match['cascade']['cpu_baseline']['value']:.3f} pairs/s")
        except Exception as ex:  # oracle missing: baseline unmeasured, not faked
            log(f"cpu baseline unavailable: {ex}")

    # HBM traffic and MFMA busy of the Schur kernel, measured now (rocprofv3
    # --pmc passes over a child run of the same C4 plan), N = 1 only
    pmc = None
    if world == 1 and rank == 0 and not args.no_pmc and args.fake_world <= 1:
        t1 = time.time()
        pmc = pmc_measure(args)
        log(f"pmc passes: {time.time() - t1:.1f}s -> {pmc}")
        if match is not None:
            t1 = time.time()
            pm = pmc_measure(args, kernel_regex="match_top2", child="--pmc-child-match")
            log(f"pmc passes (matcher): {time.time() - t1:.1f}s -> {pm}")
            if pm is not None:
                mr = match["roofline"]
                mr["traffic"] = pm["traffic"]
                mr["traffic_source"] = (f"rocprofv3 --pmc in this run: FETCH_SIZE x2 (gfx950) + WRITE_SIZE of the "
                                        f"C3 launch ({pm['launches']} launch(es))")
                # the distinct bytes a C3 launch must read at least once: every
                # image's int8 rows and key bases (each image is reused by ~499 pairs)
                mr["algorithmic_bytes_per_launch"] = args.match_frames * 4096 * (128 + 4 + 4)
                if "SQ_VALU_MFMA_BUSY_CYCLES" in pm and mr.get("per_launch_ms"):
                    mr["mfma_busy"] = pm["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * mr["per_launch_ms"] * 1e-3 * 2.4e9)
    roof = {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TF,
            "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TF,
            "traffic": None, "kernel": "schur_kernel", "per_launch_ms": schur_avg_ms,
            "per_launch_ms_basis": f"HIP events on all {schur_n} non-first Schur launches of "
                                   f"{max(3, min(args.steps, 10))} solves after the timed region",
            "algorithmic_flops_per_launch": flops,
            "flops_formula": "sum over points of 3 r (r+1) + 780 k + 30 (r = F rows of the point, "
                             "k = its observations; DESIGN.md §5)"}
    if world == 1 and rank == 0 and not args.no_pmc and args.fake_world <= 1:
        t1 = time.time()
        ks = kstats_measure(args)
        log(f"kernel-stats pass: {time.time() - t1:.1f}s -> {ks}")
        if ks is not None and ks["mean_ms"] > 0:
            # the same algorithmic flops over the profiler's mean launch time
            roof["per_launch_ms_rocprof"] = ks["mean_ms"]
            roof["achieved_rocprof"] = flops / (ks["mean_ms"] * 1e-3) / 1e12
            roof["frac_rocprof"] = roof["achieved_rocprof"] / FP64_PEAK_TF
            roof["rocprof_basis"] = (f"rocprofv3 --kernel-trace --stats in this run: mean of {ks['launches']} "
                                     f"launches of {ks['kernel']} (a child process: the C4 plan, two solves)")
    if pmc is not None:
        roof["traffic"] = pmc["traffic"]
        roof["traffic_source"] = (f"rocprofv3 --pmc in this run: FETCH_SIZE x2 (gfx950) + WRITE_SIZE, mean of "
                                  f"{pmc['launches']} launches")
        # what the pass must read: per observation uv (16 B) + slot (4 B), per
        # point X and its Jacobi scale (48 B); the RCS band it produces is < 3 MB
        roof["algorithmic_bytes_per_launch"] = 20 * sc["n_obs"] + 48 * args.n_pt
        if "SQ_VALU_MFMA_BUSY_CYCLES" in pmc and schur_avg_ms > 0:
            # busy cycles summed over the 1024 SIMDs / (SIMDs x launch time x 2.4 GHz)
            roof["mfma_busy"] = pmc["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * schur_avg_ms * 1e-3 * 2.4e9)
            if pmc.get("GRBM_GUI_ACTIVE"):
                # against the cycles the chip actually ran (GRBM_GUI_ACTIVE sums the 8 XCDs)
                roof["mfma_busy_clk"] = pmc["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * pmc["GRBM_GUI_ACTIVE"] / 8)
    elif pmc_ok:
        roof["traffic"] = pmc_traffic("schur_kernel")
        roof["traffic_source"] = "committed profiles/r*/pmc_summary.json (not measured in this run)"
    if rank == 0:
        out = {
            "metric": "BA LM-iters/sec + obs/sec, 1k cams/500k pts/5M obs; SIFT match pairs/sec",
            "value": value, "unit": "LM-iters/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"C4 BA {args.n_cam} cams / {args.n_pt} pts / {sc['n_obs']} obs, "
                                   "banded orbit visibility k=10, HuberLoss(4), gauge image 1, "
                                   "Ceres-default LM to termination per step",
                       "parallelism": f"landmark-sharded x{world}, all-reduce of the RCS",
                       "transport": transport},
            "obs_per_sec": obs_per_sec,
            "lm_iterations_per_solve": summ.iterations,
            "fake_world_exchange_estimate": fake_est,
            "rmse_initial": summ.rmse_initial, "rmse_final": summ.rmse_final,
            "roofline": roof,
            "cpu_baseline": cpu,
            "match": match,
            "ba_snavely": snav,
            "ba_pcie_inclusive": pcie,
            "loop": loop,
            "loop_fixed_writeback": loop_fixed,
            "filter": filt,
            "ba_dense_s": dense_s,
            "ba_radial3": radial3,
            "ba_radial3_percam": radial3_percam,
        }
        print(json.dumps(out))
    plan.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
