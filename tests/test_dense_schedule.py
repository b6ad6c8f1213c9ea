"""CPU: the dense RCS dataflow solve's schedule (dense_flow_plan, round 6).

dense_flow_kernel factors the reduced camera system on 64x64 tiles in an order
and with a task list the host plans once per plan: one level of nested
dissection (two chain workgroups when the camera band splits into two pieces
and a separator), the tile pattern of L with its fill, and the tasks sorted so
that every task waits only on earlier tasks and chain steps.  This test reads
the schedule through sfm_ba_dense_schedule and replays it in numpy on a random
SPD matrix with the problem's true block pattern (cameras coupled by shared
points, every camera with the intrinsics): the solution must equal
numpy.linalg.solve, the planned pattern must cover every nonzero tile, and a
round-robin replay with few workers must never stall (the kernel's
deadlock-freedom argument).  The GPU runs of the same schedule are
tests/test_seq_gpu.py, tests/test_plan_grown_gpu.py and
tests/test_ba_general_gpu.py."""
import importlib

import numpy as np
import pytest

import _helpers as H

abi = H.abi
api = importlib.import_module("3dreconstruction_amd.api")


def orbit_problem(n_img, max_len, n_intr=1, closed=False, seed=5, pts_per_img=40):
    """A sequence of images, point p seen by consecutive images first[p] ..
    (a closed orbit also links the last images with the first)."""
    rng = np.random.default_rng(seed)
    off, img = [0], []
    for c in range(n_img - 1):
        for _ in range(pts_per_img):
            n = int(rng.integers(2, max_len + 1))
            ims = [(c + k) % n_img if closed else c + k for k in range(n)]
            ims = sorted(set(i for i in ims if i < n_img))
            if len(ims) < 2:
                continue
            img += ims
            off.append(off[-1] + len(ims))
    keep = {"off": np.array(off, np.int64), "img": np.array(img, np.int32),
            "uv": rng.normal(0, 100, 2 * len(img)), "intr": (np.arange(n_img) % n_intr).astype(np.int32)}
    pr = abi.BAProblem()
    pr.n_img, pr.n_intr, pr.n_pt, pr.n_obs = n_img, n_intr, len(off) - 1, len(img)
    pr.pt_offsets, pr.obs_img = abi.ptr(keep["off"], abi.i64p), abi.ptr(keep["img"], abi.i32p)
    pr.obs_uv, pr.img_intr = abi.ptr(keep["uv"], abi.f64p), abi.ptr(keep["intr"], abi.i32p)
    pr.const_img, pr.camera_model, pr.huber_a = 0, 0, 4.0
    pr._keep = keep
    return pr


def random_problem(n_img, n_pt, seed=7):
    """Points seen by 2..5 random images: a dense camera system (the dense-S
    benchmark's shape), long left-looking sums everywhere.  One point is seen
    by every tenth image, so no camera order gives a band and the plan keeps
    image order (true_matrix's assumption)."""
    rng = np.random.default_rng(seed)
    img = list(range(0, n_img, 10))
    off = [0, len(img)]
    for _ in range(n_pt):
        ims = sorted(set(int(v) for v in rng.integers(0, n_img, int(rng.integers(2, 6)))))
        if len(ims) < 2:
            continue
        img += ims
        off.append(off[-1] + len(ims))
    keep = {"off": np.array(off, np.int64), "img": np.array(img, np.int32),
            "uv": rng.normal(0, 100, 2 * len(img)), "intr": np.zeros(n_img, np.int32)}
    pr = abi.BAProblem()
    pr.n_img, pr.n_intr, pr.n_pt, pr.n_obs = n_img, 1, len(off) - 1, len(img)
    pr.pt_offsets, pr.obs_img = abi.ptr(keep["off"], abi.i64p), abi.ptr(keep["img"], abi.i32p)
    pr.obs_uv, pr.img_intr = abi.ptr(keep["uv"], abi.f64p), abi.ptr(keep["intr"], abi.i32p)
    pr.const_img, pr.camera_model, pr.huber_a = 0, 0, 4.0
    pr._keep = keep
    return pr


def true_matrix(pr, sh, rng):
    """Random SPD S (nF x nF) with the problem's block pattern, in the plan's
    camera order (image order without the constant image: no reordering for
    these narrow bands)."""
    k = pr._keep
    nF, nb = sh["nF"], sh["nb"]
    blk = lambda i: i - 1 if i > pr.const_img else i   # noqa: E731 (const_img = 0: image i -> block i - 1)
    S = np.zeros((nF, nF))
    for p in range(pr.n_pt):
        cams = [blk(int(i)) for i in k["img"][k["off"][p]:k["off"][p + 1]] if i != pr.const_img]
        for a in cams:
            for b in cams:
                S[6 * a:6 * a + 6, 6 * b:6 * b + 6] = 1.0
    S[nb:, :nb] = 1.0   # intrinsics with every camera (one intrinsics block here)
    S[:nb, nb:] = 1.0
    S[nb:, nb:] = 1.0
    V = np.tril(rng.normal(0, 0.1, (nF, nF)) * S)
    V = V + V.T
    return V + np.eye(nF) * (np.abs(V).sum(1).max() + 1.0)


def replay(sh, meta, S, rhs, workers):
    nt = sh["nt"]
    n = 64 * nt
    perm, prev, info = meta[:nt], meta[nt:2 * nt], meta[2 * nt:3 * nt]
    c0 = list(meta[4 * nt:4 * nt + meta[6 * nt]])
    c1 = list(meta[5 * nt:5 * nt + meta[6 * nt + 1]])
    ntask = sh["tasks"]
    tasks = meta[6 * nt + 2:6 * nt + 2 + ntask]
    nz = np.frombuffer(meta[6 * nt + 2 + ntask:].astype("<i4").tobytes(), np.uint8)[:nt * nt].reshape(nt, nt)
    A = np.eye(n)
    A[:S.shape[0], :S.shape[0]] = S
    b = np.zeros(n)
    b[:len(rhs)] = rhs
    idx = np.concatenate([np.arange(64 * p, 64 * p + 64) for p in perm])
    Ap, bp = A[np.ix_(idx, idx)], b[idx]
    T = lambda M, i, j: M[64 * i:64 * i + 64, 64 * j:64 * j + 64]  # noqa: E731
    for i in range(nt):
        for j in range(i + 1):
            assert nz[i, j] or not T(Ap, i, j).any(), ("pattern misses tile", i, j)
    Lt, X, At, y, x, avail = {}, {}, {}, {}, {}, set()
    chains, cpos, Xp = [c0, c1], [0, 0], [None, None]
    queue = [list(range(w, ntask, workers)) for w in range(min(workers, ntask))]
    ptr = [0] * len(queue)
    moved = True
    while moved:
        moved = False
        for c in range(2):
            ch = chains[c]
            if cpos[c] >= len(ch):
                continue
            q = cpos[c]
            k, p, inf = ch[q], prev[ch[q]], info[ch[q]]
            if (inf & 2 and ("D", k) not in avail) or (inf & 4 and ("S", k) not in avail):
                continue
            Akk = At.get((k, k), T(Ap, k, k))
            if inf & 1:
                L = At.get((k, p), T(Ap, k, p)) @ Xp[c].T
                Lt[(k, p)] = L
                avail |= {("L", k, p), ("X", p)}
                Akk = Akk - L @ L.T
            X[k] = Xp[c] = np.linalg.inv(np.linalg.cholesky(np.tril(Akk) + np.tril(Akk, -1).T))
            nxt = ch[q + 1] if q + 1 < len(ch) else -1
            if nxt < 0 or not info[nxt] & 1:
                avail.add(("X", k))
            cpos[c] += 1
            moved = True
        for w in range(len(queue)):
            if ptr[w] >= len(queue[w]):
                continue
            code = int(tasks[queue[w][ptr[w]]])
            kind, i, j = code >> 24, (code >> 12) & 0xfff, code & 0xfff
            if kind <= 2:
                diag = kind == 0
                excl = prev[i] if diag and info[i] & 1 else -1
                ms = [m for m in range(i if diag else j) if m != excl and nz[i, m] and (diag or nz[j, m])]
                # a D / S task forms a terms-free L_im (pattern bit 1) itself from X_m
                local = {m for m in ms if kind != 2 and nz[i, m] & 2}
                if not all((("X", m) if m in local else ("L", i, m)) in avail and ("L", j, m) in avail
                           for m in ms if j != i or m not in local) or \
                        not all(("X", m) in avail for m in local):
                    continue
                if kind == 2 and ("X", j) not in avail:
                    continue
                acc = T(Ap, i, j).copy()
                for m in ms:
                    Li = T(Ap, i, m) @ X[m].T if m in local else Lt[(i, m)]
                    acc -= Li @ (Li if j == i else Lt[(j, m)]).T
                if kind == 2:
                    Lt[(i, j)] = acc @ X[j].T
                    avail.add(("L", i, j))
                else:
                    At[(i, j)] = acc
                    avail.add(("D" if diag else "S", i))
            elif kind == 3:
                ms = [m for m in range(j) if nz[j, m]]
                if ("X", j) not in avail or not all(("L", j, m) in avail and ("y", m) in avail for m in ms):
                    continue
                y[j] = X[j] @ (bp[64 * j:64 * j + 64] - sum((Lt[(j, m)] @ y[m] for m in ms), np.zeros(64)))
                avail.add(("y", j))
            else:
                rs = [r for r in range(i + 1, nt) if nz[r, i]]
                if ("X", i) not in avail or ("y", i) not in avail or \
                        not all(("L", r, i) in avail and ("x", r) in avail for r in rs):
                    continue
                x[i] = X[i].T @ (y[i] - sum((Lt[(r, i)].T @ x[r] for r in rs), np.zeros(64)))
                avail.add(("x", i))
            ptr[w] += 1
            moved = True
    assert all(ptr[w] == len(queue[w]) for w in range(len(queue))), "a worker stalled"
    assert cpos == [len(c0), len(c1)], "a chain stalled"
    out = np.zeros(n)
    for k in range(nt):
        out[64 * perm[k]:64 * perm[k] + 64] = x[k]
    return out[:S.shape[0]]


@pytest.mark.parametrize("n_img,max_len,closed,chains", [
    (300, 14, False, 2),   # the C5 loop's shape: band of 13 blocks, nested dissection
    (130, 12, False, 2),
    (60, 14, False, 1),    # too short to split
    (120, 14, True, 1),    # closed orbit: the band wraps, no split
])
def test_dense_schedule_replays_to_the_solution(n_img, max_len, closed, chains):
    pr = orbit_problem(n_img, max_len, closed=closed)
    sh, meta = api.ba_dense_schedule(pr)
    assert sh["flow"] == 1 and sh["chains"] == chains, sh
    rng = np.random.default_rng(n_img)
    S = true_matrix(pr, sh, rng)
    rhs = rng.normal(size=S.shape[0])
    ref = np.linalg.solve(S, rhs)
    for workers in (254, 5, 1):
        got = replay(sh, meta, S, rhs, workers)
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-11 * np.abs(ref).max())


def test_dense_schedule_random_visibility():
    """A dense camera system (38 block columns, sums of up to 37 terms, one
    chain): the replay solves it and never stalls with 254, 3 or 1 workers."""
    pr = random_problem(400, 3000)
    sh, meta = api.ba_dense_schedule(pr)
    assert sh["flow"] == 1 and sh["chains"] == 1 and sh["nt"] == 38, sh
    rng = np.random.default_rng(11)
    S = true_matrix(pr, sh, rng)
    rhs = rng.normal(size=S.shape[0])
    ref = np.linalg.solve(S, rhs)
    for workers in (254, 3, 1):
        got = replay(sh, meta, S, rhs, workers)
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-10 * np.abs(ref).max())


def percam_problem(n_img, max_len, closed, seed=9, pts_per_img=30):
    """RADIAL3 with one intrinsics block per image (reconstruction()'s
    grouping): the intrinsics arrow is as wide as the camera band and itself
    banded.  Observations as orbit_problem's."""
    pr = orbit_problem(n_img, max_len, n_intr=n_img, closed=closed, seed=seed, pts_per_img=pts_per_img)
    pr.camera_model = abi.SFM_CAM_RADIAL3
    return pr


def percam_matrix(pr, sh, rng, iw=6):
    """Random SPD S with the per-camera problem's exact block pattern: every
    pair of the point's camera blocks and intrinsics blocks couples."""
    k = pr._keep
    nF, nb = sh["nF"], sh["nb"]
    S = np.zeros((nF, nF))
    for p in range(pr.n_pt):
        ims = [int(i) for i in k["img"][k["off"][p]:k["off"][p + 1]]]
        rows = [6 * (i - 1) for i in ims if i != pr.const_img] + [nb + iw * int(k["intr"][i]) for i in ims]
        for a in rows:
            for b in rows:
                S[a:a + 6, b:b + 6] = 1.0
    V = np.tril(rng.normal(0, 0.1, (nF, nF)) * S)
    V = V + V.T
    return V + np.eye(nF) * (np.abs(V).sum(1).max() + 1.0)


@pytest.mark.parametrize("n_img,max_len", [(200, 10), (150, 6)])
def test_dense_schedule_banded_arrow(n_img, max_len):
    """One intrinsics block per camera: the tiles are ordered by Cuthill-McKee
    over the exact tile pattern (the reduce's targets) and split over two
    chains; the replay solves the system with that pattern and never stalls."""
    pr = percam_problem(n_img, max_len, False)   # (open: the plan keeps image order, percam_matrix's)
    sh, meta = api.ba_dense_schedule(pr)
    nt = sh["nt"]
    assert sh["flow"] == 1 and sh["chains"] == 2, sh
    # intrinsics tiles (natural index >= nb / 64) among the first columns: the
    # arrow is ordered into the band, not left to the end of chain 0
    assert any(int(p) >= sh["nb"] // 64 for p in meta[:nt // 2]), meta[:nt]
    rng = np.random.default_rng(n_img)
    S = percam_matrix(pr, sh, rng)
    rhs = rng.normal(size=S.shape[0])
    ref = np.linalg.solve(S, rhs)
    for workers in (254, 3, 1):
        got = replay(sh, meta, S, rhs, workers)
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-10 * np.abs(ref).max())


def test_dense_schedule_absent_for_band_problems():
    sh, meta = api.ba_dense_schedule(orbit_problem(200, 8))   # band of 7 blocks: the BCR solver
    assert sh["flow"] == 0 and len(meta) == 0
