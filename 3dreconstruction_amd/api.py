"""Thin numpy wrappers over libsfmcore.so (ctypes) for tests and bench.py.

Every call goes through the C-ABI in include/sfmcore.h; there is no Python
compute path and no fallback: if the library or a gfx950 device is missing,
these raise.
"""
import ctypes as C

import numpy as np

from . import _abi as abi


class SfmError(RuntimeError):
    def __init__(self, code, where):
        lib = abi.load()
        msg = lib.sfm_last_error().decode(errors="replace")
        super().__init__(f"{where} failed with {code}: {msg}")
        self.code = code


def _check(rc, where):
    if rc != abi.SFM_OK:
        raise SfmError(rc, where)


class Context:
    """sfm_ctx: one HIP device (+ RCCL communicator when world_size > 1).

    allreduce: optional callable (numpy float64 array, op) -> None reducing the
    array in place across ranks (op 0 sum, 1 max); replaces RCCL, e.g. with a
    torch.distributed gloo group."""

    def __init__(self, device=0, rank=0, world_size=1, comm_id=None, allreduce=None, flags=0):
        self.lib = abi.load()
        o = abi.CtxOpts()
        o.device, o.rank, o.world_size, o.flags = device, rank, world_size, flags
        self._id = None
        self._hook = None
        if comm_id is not None:
            self._id = (C.c_uint8 * 128).from_buffer_copy(bytes(comm_id))
            o.comm_id = C.cast(self._id, abi.u8p)
        if allreduce is not None:
            import numpy as np

            def hook(user, buf, n, op):
                try:
                    allreduce(np.ctypeslib.as_array(buf, shape=(n,)), int(op))
                    return 0
                except Exception:
                    return -1

            self._hook = abi.ALLREDUCE_HOOK(hook)
            o.allreduce = C.cast(self._hook, C.c_void_p)
        h = C.c_void_p()
        _check(self.lib.sfm_ctx_create(C.byref(o), C.byref(h)), "sfm_ctx_create")
        self.h = h
        self._children = []

    def _adopt(self, child):
        import weakref
        self._children.append(weakref.ref(child))

    def synchronize(self):
        _check(self.lib.sfm_ctx_synchronize(self.h), "sfm_ctx_synchronize")

    def close(self):
        if self.h:
            for r in self._children:  # plans must die before their context
                c = r()
                if c is not None:
                    c.close()
            self.lib.sfm_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id():
    lib = abi.load()
    buf = (C.c_uint8 * 128)()
    _check(lib.sfm_comm_unique_id(buf), "sfm_comm_unique_id")
    return bytes(buf)


def match_dense(ctx, a, b, mode=abi.SFM_MATCH_RATIO, ratio=0.8):
    a = np.ascontiguousarray(a, np.uint8).reshape(-1, 128)
    b = np.ascontiguousarray(b, np.uint8).reshape(-1, 128)
    n_out = len(a) if mode == abi.SFM_MATCH_MUTUAL else len(b)
    idx = np.zeros(max(n_out, 1), np.int32)
    d2 = np.zeros(max(n_out, 1), np.int32)
    o = abi.MatchOptions(mode, ratio)
    _check(ctx.lib.sfm_match_dense(ctx.h, abi.ptr(a, abi.u8p), len(a), abi.ptr(b, abi.u8p), len(b),
                                   C.byref(o), abi.ptr(idx, abi.i32p), abi.ptr(d2, abi.i32p)),
           "sfm_match_dense")
    return idx[:n_out], d2[:n_out]


def match_dense_f32(ctx, a, b, mode=abi.SFM_MATCH_RATIO, ratio=0.8):
    """sfm_match_dense_f32: float descriptors (cv::Mat CV_32F); returns
    (idx, squared distance as float32, -1 where unmatched)."""
    a = np.ascontiguousarray(a, np.float32).reshape(-1, 128)
    b = np.ascontiguousarray(b, np.float32).reshape(-1, 128)
    n_out = len(a) if mode == abi.SFM_MATCH_MUTUAL else len(b)
    idx = np.zeros(max(n_out, 1), np.int32)
    d2 = np.zeros(max(n_out, 1), np.float32)
    o = abi.MatchOptions(mode, ratio)
    _check(ctx.lib.sfm_match_dense_f32(ctx.h, abi.ptr(a, abi.f32p), len(a), abi.ptr(b, abi.f32p), len(b),
                                       C.byref(o), abi.ptr(idx, abi.i32p), abi.ptr(d2, abi.f32p)),
           "sfm_match_dense_f32")
    return idx[:n_out], d2[:n_out]


class MatchPlan:
    """Resident descriptor collection for all-pairs matching (uint8, or float32
    through sfm_match_plan_create_f32: fetch() then returns float distances)."""

    def __init__(self, ctx, desc, offsets):
        self.ctx = ctx
        self.f32 = np.asarray(desc).dtype == np.float32
        offsets = np.ascontiguousarray(offsets, np.int64)
        self.n_img = len(offsets) - 1
        h = C.c_void_p()
        if self.f32:
            desc = np.ascontiguousarray(desc, np.float32).reshape(-1, 128)
            _check(ctx.lib.sfm_match_plan_create_f32(ctx.h, abi.ptr(desc, abi.f32p),
                                                     abi.ptr(offsets, abi.i64p), self.n_img, C.byref(h)),
                   "sfm_match_plan_create_f32")
        else:
            desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 128)
            _check(ctx.lib.sfm_match_plan_create(ctx.h, abi.ptr(desc, abi.u8p),
                                                 abi.ptr(offsets, abi.i64p), self.n_img, C.byref(h)),
                   "sfm_match_plan_create")
        self.h = h
        self.n_pairs = 0
        ctx._adopt(self)

    def run(self, pairs, mode=abi.SFM_MATCH_RATIO, ratio=0.8, count=True):
        pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
        self.n_pairs = len(pairs)
        o = abi.MatchOptions(mode, ratio)
        tot = C.c_int64()
        _check(self.ctx.lib.sfm_match_plan_run(self.h, abi.ptr(pairs, abi.i32p), len(pairs),
                                               C.byref(o), C.byref(tot) if count else None),
               "sfm_match_plan_run")
        return tot.value if count else None

    def fetch(self):
        counts = np.zeros(max(self.n_pairs, 1), np.int64)
        fetch = self.ctx.lib.sfm_match_plan_fetch_f32 if self.f32 else self.ctx.lib.sfm_match_plan_fetch
        _check(fetch(self.h, abi.ptr(counts, abi.i64p), None, None, None), "sfm_match_plan_fetch")
        counts = counts[:self.n_pairs]
        tot = int(counts.sum())
        i = np.zeros(max(tot, 1), np.uint32)
        j = np.zeros(max(tot, 1), np.uint32)
        if self.f32:
            d = np.zeros(max(tot, 1), np.float32)
            _check(self.ctx.lib.sfm_match_plan_fetch_f32(self.h, abi.ptr(counts, abi.i64p),
                                                         abi.ptr(i, abi.u32p), abi.ptr(j, abi.u32p),
                                                         abi.ptr(d, abi.f32p)), "sfm_match_plan_fetch_f32")
        else:
            d = np.zeros(max(tot, 1), np.int32)
            _check(self.ctx.lib.sfm_match_plan_fetch(self.h, abi.ptr(counts, abi.i64p),
                                                     abi.ptr(i, abi.u32p), abi.ptr(j, abi.u32p),
                                                     abi.ptr(d, abi.i32p)), "sfm_match_plan_fetch")
        return counts, i[:tot], j[:tot], d[:tot]

    def cascade_index(self, pairs):
        """Hash tables for the images of `pairs` (SFM_MATCH_CASCADE); later
        cascade runs over any part of that list reuse them."""
        pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
        _check(self.ctx.lib.sfm_match_plan_cascade_index(self.h, abi.ptr(pairs, abi.i32p),
                                                         len(pairs)), "sfm_match_plan_cascade_index")

    def digest(self):
        v = C.c_uint64()
        _check(self.ctx.lib.sfm_match_plan_digest(self.h, C.byref(v)), "sfm_match_plan_digest")
        return v.value

    def last_ms(self):
        ms = C.c_double()
        n = C.c_int64()
        _check(self.ctx.lib.sfm_match_plan_get_last_ms(self.h, C.byref(ms), C.byref(n)),
               "sfm_match_plan_get_last_ms")
        return ms.value, n.value

    def close(self):
        if self.h:
            self.ctx.lib.sfm_match_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _mix64(z):
    z = np.uint64(z)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def match_digest(counts, i, j, d):
    """Host restatement of the device digest (order-independent)."""
    tot = np.uint64(0)
    off = 0
    with np.errstate(over="ignore"):
        for p, c in enumerate(counts):
            h = np.uint64(0)
            for k in range(off, off + int(c)):
                key = (np.uint64(i[k]) << np.uint64(32)) | np.uint64(j[k])
                h = h + _mix64(key ^ (np.uint64(np.uint32(d[k])) << np.uint64(21)))
            off += int(c)
            tot = tot + _mix64(h + np.uint64(0x9E3779B97F4A7C15) * np.uint64(p + 1))
    return int(tot)


def exhaustive_pairs(n):
    lib = abi.load()
    m = n * (n - 1) // 2
    out = np.zeros(max(2 * m, 2), np.int32)
    _check(lib.sfm_exhaustive_pairs(n, abi.ptr(out, abi.i32p)), "sfm_exhaustive_pairs")
    return out[:2 * m].reshape(-1, 2)


def synth_descriptors(n_img, n_kp, seed=0xC3):
    lib = abi.load()
    d = np.zeros(max(n_img * n_kp * 128, 1), np.uint8)
    _check(lib.sfm_synth_descriptors(n_img, n_kp, seed, abi.ptr(d, abi.u8p)),
           "sfm_synth_descriptors")
    return d[:n_img * n_kp * 128].reshape(-1, 128)


def ba_describe(problem, rank=0, world=1):
    """[cpu] The planner's structure for a problem (sfm_ba_describe)."""
    lib = abi.load()
    out = abi.BAPlanShape()
    _check(lib.sfm_ba_describe(C.byref(problem), rank, world, C.byref(out)), "sfm_ba_describe")
    return out


def ba_grown_digest(prev, problem):
    """[cpu] (fresh digest, grown digest, reused sorted points) of `problem`
    planned from scratch and grown from `prev`'s plan (sfm_ba_grown_digest)."""
    lib = abi.load()
    df, dg, r = C.c_uint64(), C.c_uint64(), C.c_int64()
    _check(lib.sfm_ba_grown_digest(C.byref(prev), C.byref(problem), C.byref(df), C.byref(dg), C.byref(r)),
           "sfm_ba_grown_digest")
    return df.value, dg.value, r.value


def ba_dense_schedule(problem):
    """[cpu] The dense dataflow solve's schedule for `problem`
    (sfm_ba_dense_schedule): (shape dict, int32 array); the array is empty
    when the dataflow solve does not run."""
    lib = abi.load()
    n = C.c_int64()
    shape = np.zeros(7, np.int32)
    _check(lib.sfm_ba_dense_schedule(C.byref(problem), None, 0, C.byref(n), shape.ctypes.data_as(abi.i32p)),
           "sfm_ba_dense_schedule")
    meta = np.zeros(max(n.value, 1), np.int32)
    _check(lib.sfm_ba_dense_schedule(C.byref(problem), meta.ctypes.data_as(abi.i32p), n.value, C.byref(n),
                                     shape.ctypes.data_as(abi.i32p)), "sfm_ba_dense_schedule")
    keys = ("nt", "chains", "tasks", "flow", "nF", "nb", "D")
    return dict(zip(keys, (int(v) for v in shape))), meta[:n.value]


class BAPlan:
    """Resident BA problem (sfm_ba_plan): upload once, run many times."""

    def __init__(self, ctx, problem, extr, intr, X):
        self.ctx = ctx
        self._keep = (problem, extr, intr, X)
        h = C.c_void_p()
        _check(ctx.lib.sfm_ba_plan_create(ctx.h, C.byref(problem), abi.ptr(extr, abi.f64p),
                                          abi.ptr(intr, abi.f64p), abi.ptr(X, abi.f64p),
                                          C.byref(h)), "sfm_ba_plan_create")
        self.h = h
        self.shape = (len(extr), len(intr), len(X))
        ctx._adopt(self)

    def run(self, opts=None, check=True):
        o = opts or abi.default_options()
        s = abi.BASummary()
        rc = self.ctx.lib.sfm_ba_plan_run(self.h, C.byref(o), C.byref(s))
        if check and rc not in (abi.SFM_OK, abi.SFM_ERR_SOLVER):
            _check(rc, "sfm_ba_plan_run")
        return rc, s

    def download(self):
        e, i, x = (np.zeros(n) for n in self.shape)
        _check(self.ctx.lib.sfm_ba_plan_download(self.h, abi.ptr(e, abi.f64p), abi.ptr(i, abi.f64p),
                                                 abi.ptr(x, abi.f64p)), "sfm_ba_plan_download")
        return e, i, x

    def info(self):
        inf = abi.BAPlanInfo()
        _check(self.ctx.lib.sfm_ba_plan_get_info(self.h, C.byref(inf)), "sfm_ba_plan_get_info")
        return inf

    def trace(self, cap=256):
        tr = (abi.BAIter * cap)()
        n = C.c_int32()
        _check(self.ctx.lib.sfm_ba_plan_get_trace(self.h, tr, cap, C.byref(n)),
               "sfm_ba_plan_get_trace")
        return [tr[k] for k in range(n.value)]

    def close(self):
        if self.h:
            self.ctx.lib.sfm_ba_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ba_solve(ctx, problem, extr, intr, X, opts=None):
    """sfm_ba_solve: in-place update of extr/intr/X when the solution is usable."""
    o = opts or abi.default_options()
    s = abi.BASummary()
    rc = ctx.lib.sfm_ba_solve(ctx.h, C.byref(problem), abi.ptr(extr, abi.f64p),
                              abi.ptr(intr, abi.f64p), abi.ptr(X, abi.f64p), C.byref(o),
                              C.byref(s))
    return rc, s


def ba_cache_stats(ctx):
    """(reused, grown, fresh) plan counts of sfm_ba_solve on this context."""
    r, g, f = C.c_int64(), C.c_int64(), C.c_int64()
    _check(ctx.lib.sfm_ba_cache_stats(ctx.h, C.byref(r), C.byref(g), C.byref(f)), "sfm_ba_cache_stats")
    return r.value, g.value, f.value


def ba_cache_clear(ctx):
    _check(ctx.lib.sfm_ba_cache_clear(ctx.h), "sfm_ba_cache_clear")


def ba_partition(problem, world_size):
    lib = abi.load()
    order = np.zeros(max(problem.n_pt, 1), np.int64)
    bounds = np.zeros(world_size + 1, np.int64)
    _check(lib.sfm_ba_partition(C.byref(problem), world_size, abi.ptr(order, abi.i64p),
                                abi.ptr(bounds, abi.i64p)), "sfm_ba_partition")
    return order[:problem.n_pt], bounds


# ---------------------------------------------------------------------------
# incremental SequentialActuator loop (config C5)
# ---------------------------------------------------------------------------
def seq_default_options():
    o = abi.SeqOptions()
    abi.load().sfm_seq_default_options(C.byref(o))
    return o


class OrbitSequence:
    """[cpu] The synthetic closed-orbit image sequence (sfm_synth_orbit_image)."""

    def __init__(self, n_img=300, n_landmarks=60000, n_clutter=1000, track_mean=10.0,
                 detect_prob=0.95, noise_px=0.5, desc_noise_dims=24, desc_noise_amp=3,
                 prior_rot=2e-4, prior_t=1e-3, seed=0x5F3D0005):
        c = abi.SynthOrbitConfig()
        c.n_img, c.n_clutter, c.n_landmarks = n_img, n_clutter, n_landmarks
        c.track_mean, c.detect_prob, c.noise_px = track_mean, detect_prob, noise_px
        c.desc_noise_dims, c.desc_noise_amp = desc_noise_dims, desc_noise_amp
        c.prior_rot, c.prior_t, c.seed = prior_rot, prior_t, seed
        self.cfg = c
        self.n_img = n_img

    def image(self, k, gt=False):
        """dict(kp [n,2] f64, desc [n,128] u8, prior [6], landmark [n] (gt))"""
        lib = abi.load()
        n = C.c_int32()
        _check(lib.sfm_synth_orbit_image(C.byref(self.cfg), k, C.byref(n), None, None, None, None,
                                         None), "sfm_synth_orbit_image")
        kp = np.zeros((n.value, 2))
        d = np.zeros((max(n.value, 1), 128), np.uint8)
        prior = np.zeros(6)
        lm = np.zeros(max(n.value, 1), np.int64)
        _check(lib.sfm_synth_orbit_image(C.byref(self.cfg), k, C.byref(n), abi.ptr(kp, abi.f64p),
                                         abi.ptr(d, abi.u8p), abi.ptr(prior, abi.f64p),
                                         abi.ptr(lm, abi.i64p), None), "sfm_synth_orbit_image")
        out = {"kp": kp, "desc": d[:n.value], "prior": prior}
        if gt:
            out["landmark"] = lm[:n.value]
        return out

    def gt_points(self):
        lib = abi.load()
        n = C.c_int32()
        X = np.zeros(3 * max(self.cfg.n_landmarks, 1))
        _check(lib.sfm_synth_orbit_image(C.byref(self.cfg), 0, C.byref(n), None, None, None, None,
                                         abi.ptr(X, abi.f64p)), "sfm_synth_orbit_image")
        return X[:3 * self.cfg.n_landmarks].reshape(-1, 3)


def seq_image(img):
    """numpy image dict -> SeqImage (keeps the arrays referenced)."""
    si = abi.SeqImage()
    kp = np.ascontiguousarray(img["kp"], np.float64)
    d = np.ascontiguousarray(img["desc"], np.uint8)
    si.n_kp = len(kp)
    si.kp_xy = abi.ptr(kp, abi.f64p)
    si.desc = abi.ptr(d, abi.u8p)
    for a in range(6):
        si.pose_prior[a] = float(img["prior"][a])
    si._keep = (kp, d)
    return si


class _SeqCalls:
    """init / add / bundle_adjust / step / matches / world over the sfm_seq_*
    (product) or orc_seq_* (oracle, tests only) entry points."""

    def _f(self, name):
        return getattr(self.lib, self.prefix + name)

    def init(self, a, b):
        _check(self._f("init")(self.h, C.byref(seq_image(a)), C.byref(seq_image(b))), self.prefix + "init")

    def add(self, img):
        kept = C.c_int32()
        _check(self._f("add_image")(self.h, C.byref(seq_image(img)), C.byref(kept)), self.prefix + "add_image")
        return bool(kept.value)

    def bundle_adjust(self):
        s = abi.BASummary()
        _check(self._f("bundle_adjust")(self.h, C.byref(s)), self.prefix + "bundle_adjust")
        return s

    def step(self):
        st = abi.SeqStep()
        _check(self._f("last_step")(self.h, C.byref(st)), self.prefix + "last_step")
        return st

    def matches(self, which):
        n = C.c_int64()
        self._f("matches")(self.h, which, None, None, None, 0, C.byref(n))
        q = np.zeros(max(n.value, 1), np.int32)
        t = np.zeros_like(q)
        d = np.zeros(len(q), np.float32)
        _check(self._f("matches")(self.h, which, abi.ptr(q, abi.i32p), abi.ptr(t, abi.i32p),
                                  abi.ptr(d, abi.f32p), n.value, C.byref(n)), self.prefix + "matches")
        return q[:n.value], t[:n.value], d[:n.value]

    def world(self):
        n_pts, n_img = C.c_int64(), C.c_int32()
        self._f("world")(self.h, None, None, 0, C.byref(n_pts), None, 0, C.byref(n_img), None)
        X = np.zeros(3 * max(n_pts.value, 1))
        nobs = np.zeros(max(n_pts.value, 1), np.int64)
        poses = np.zeros(6 * max(n_img.value, 1))
        intr = np.zeros(4)
        _check(self._f("world")(self.h, abi.ptr(X, abi.f64p), abi.ptr(nobs, abi.i64p), n_pts.value,
                                C.byref(n_pts), abi.ptr(poses, abi.f64p), n_img.value, C.byref(n_img),
                                abi.ptr(intr, abi.f64p)), self.prefix + "world")
        return {"X": X[:3 * n_pts.value].reshape(-1, 3), "n_obs": nobs[:n_pts.value],
                "poses": poses[:6 * n_img.value].reshape(-1, 6), "intr": intr}

    def observations(self):
        """(image sequence index [n], uv [n, 2]) of every observation, points
        in index order (counts: world()["n_obs"])"""
        n = C.c_int64()
        self._f("observations")(self.h, None, None, 0, C.byref(n))
        img = np.zeros(max(n.value, 1), np.int32)
        uv = np.zeros((max(n.value, 1), 2))
        _check(self._f("observations")(self.h, abi.ptr(img, abi.i32p), abi.ptr(uv, abi.f64p), n.value,
                                       C.byref(n)), self.prefix + "observations")
        return img[:n.value], uv[:n.value]

    def close(self):
        if self.h:
            self._f("destroy")(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SeqLoop(_SeqCalls):
    """SequentialActuator on the GPU (sfm_seq_*)."""

    def __init__(self, ctx, opts=None):
        self.ctx, self.lib, self.prefix = ctx, ctx.lib, "sfm_seq_"
        o = opts or seq_default_options()
        h = C.c_void_p()
        _check(self.lib.sfm_seq_create(ctx.h, C.byref(o), C.byref(h)), "sfm_seq_create")
        self.h = h
        ctx._adopt(self)


# ---------------------------------------------------------------------------
# file-staged sparseBuilder flow (OpenMVG stage-boundary formats)
# ---------------------------------------------------------------------------
def _b(path):
    return str(path).encode()


def mvg_load_views(path):
    """sfm_data.json VIEWS -> list of dicts sorted by id_view."""
    lib = abi.load()
    n = C.c_int32()
    _check(lib.sfm_mvg_load_views(_b(path), None, 0, C.byref(n)), "sfm_mvg_load_views")
    v = (abi.MvgView * max(n.value, 1))()
    _check(lib.sfm_mvg_load_views(_b(path), v, n.value, C.byref(n)), "sfm_mvg_load_views")
    return [{"id_view": x.id_view, "id_intrinsic": x.id_intrinsic, "id_pose": x.id_pose,
             "width": x.width, "height": x.height, "img_path": x.img_path.decode()}
            for x in v[:n.value]]


def mvg_check_describer(path):
    _check(abi.load().sfm_mvg_check_describer(_b(path)), "sfm_mvg_check_describer")


def mvg_read_desc(path):
    lib = abi.load()
    n = C.c_int64()
    _check(lib.sfm_mvg_read_desc(_b(path), None, 0, C.byref(n)), "sfm_mvg_read_desc")
    d = np.zeros((max(n.value, 1), 128), np.uint8)
    _check(lib.sfm_mvg_read_desc(_b(path), abi.ptr(d, abi.u8p), n.value, C.byref(n)),
           "sfm_mvg_read_desc")
    return d[:n.value]


def mvg_write_desc(path, desc):
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 128)
    _check(abi.load().sfm_mvg_write_desc(_b(path), abi.ptr(d, abi.u8p), d.shape[0]),
           "sfm_mvg_write_desc")


def mvg_read_feat(path):
    lib = abi.load()
    n = C.c_int64()
    _check(lib.sfm_mvg_read_feat(_b(path), None, 0, C.byref(n)), "sfm_mvg_read_feat")
    f = np.zeros((max(n.value, 1), 4), np.float32)
    _check(lib.sfm_mvg_read_feat(_b(path), f.ctypes.data_as(C.POINTER(C.c_float)), n.value,
                                 C.byref(n)), "sfm_mvg_read_feat")
    return f[:n.value]


def mvg_load_pairs(path, n_views):
    lib = abi.load()
    n = C.c_int64()
    _check(lib.sfm_mvg_load_pairs(_b(path), n_views, None, 0, C.byref(n)), "sfm_mvg_load_pairs")
    p = np.zeros((max(n.value, 1), 2), np.int32)
    _check(lib.sfm_mvg_load_pairs(_b(path), n_views, abi.ptr(p, abi.i32p), n.value, C.byref(n)),
           "sfm_mvg_load_pairs")
    return p[:n.value]


def mvg_save_pairs(path, pairs):
    p = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
    _check(abi.load().sfm_mvg_save_pairs(_b(path), abi.ptr(p, abi.i32p), p.shape[0]),
           "sfm_mvg_save_pairs")


def mvg_save_matches(path, matches):
    """matches: {(I, J): int array [n, 2] of (i, j)} -> PairWiseMatches file."""
    keys = sorted(matches)
    pairs = np.array(keys, np.int32).reshape(-1, 2)
    counts = np.array([len(matches[k]) for k in keys], np.int64)
    ij = np.concatenate([np.asarray(matches[k], np.uint32).reshape(-1, 2) for k in keys]) \
        if keys else np.zeros((0, 2), np.uint32)
    i = np.ascontiguousarray(ij[:, 0])
    j = np.ascontiguousarray(ij[:, 1])
    _check(abi.load().sfm_mvg_save_matches(_b(path), abi.ptr(pairs, abi.i32p), len(keys),
                                           abi.ptr(counts, abi.i64p), abi.ptr(i, abi.u32p),
                                           abi.ptr(j, abi.u32p)), "sfm_mvg_save_matches")


def mvg_load_matches(path):
    """PairWiseMatches file -> {(I, J): uint32 array [n, 2]} (map order)."""
    lib = abi.load()
    npair, nm = C.c_int64(), C.c_int64()
    _check(lib.sfm_mvg_load_matches(_b(path), None, None, None, None, 0, 0, C.byref(npair),
                                    C.byref(nm)), "sfm_mvg_load_matches")
    pairs = np.zeros((max(npair.value, 1), 2), np.int32)
    counts = np.zeros(max(npair.value, 1), np.int64)
    i = np.zeros(max(nm.value, 1), np.uint32)
    j = np.zeros(max(nm.value, 1), np.uint32)
    _check(lib.sfm_mvg_load_matches(_b(path), abi.ptr(pairs, abi.i32p), abi.ptr(counts, abi.i64p),
                                    abi.ptr(i, abi.u32p), abi.ptr(j, abi.u32p), npair.value,
                                    nm.value, C.byref(npair), C.byref(nm)), "sfm_mvg_load_matches")
    out, off = {}, 0
    for k in range(npair.value):
        c = int(counts[k])
        out[(int(pairs[k, 0]), int(pairs[k, 1]))] = np.stack([i[off:off + c], j[off:off + c]], 1)
        off += c
    return out


def sparse_match_pair(matches_dir):
    """sparseBuilder::matchPair(): writes <matches_dir>/pairs.bin."""
    _check(abi.load().sfm_sparse_match_pair(_b(matches_dir)), "sfm_sparse_match_pair")


def sparse_match(ctx, matches_dir, mode=abi.SFM_MATCH_CASCADE, ratio=0.8, force=False, dedup_xy=True):
    """sparseBuilder::match(), file-staged, on the GPU matcher.  The default
    mode is the reference's "AUTO" (cascade hashing, sparseBuilder.cpp:814,
    911-914); SFM_MATCH_RATIO is its "BRUTEFORCEL2" (:919-921)."""
    o = abi.SparseMatchOpts()
    o.mode, o.ratio, o.force, o.dedup_xy = mode, ratio, int(force), int(dedup_xy)
    st = abi.SparseMatchStats()
    _check(ctx.lib.sfm_sparse_match(ctx.h, _b(matches_dir), C.byref(o), C.byref(st)),
           "sfm_sparse_match")
    return {"n_views": st.n_views, "n_pairs_in": st.n_pairs_in, "n_pairs_out": st.n_pairs_out,
            "n_matches": st.n_matches, "reloaded": bool(st.reloaded)}


# ---- geometric filter (GeometricFilter_FMatrix_AC) ----------
def fmatrix_opts(precision=4.0, max_iterations=2048):
    o = abi.FMatrixOpts()
    o.precision, o.max_iterations = precision, max_iterations
    return o


def _fmatrix_inputs(xy_list, wh):
    counts = np.array([len(x) for x in xy_list], np.int64)
    off = np.zeros(len(xy_list) + 1, np.int64)
    off[1:] = np.cumsum(counts)
    xy = np.ascontiguousarray(np.concatenate([np.asarray(x, np.float64).reshape(-1, 4) for x in xy_list])
                              if len(xy_list) and off[-1] else np.zeros((1, 4)), np.float64)
    wh = np.ascontiguousarray(np.asarray(wh, np.int32).reshape(-1, 4))
    return off, xy, wh


def _fmatrix_outputs(off, res, inl):
    out = []
    for q in range(len(off) - 1):
        r = res[q]
        out.append({"F": np.array(r.F[:]).reshape(3, 3), "error_max": r.error_max, "min_nfa": r.min_nfa,
                    "n_inliers": r.n_inliers, "iterations": r.iterations,
                    "inliers": inl[off[q]:off[q] + r.n_inliers].copy()})
    return out


def fmatrix_ac(ctx, xy_list, wh, opts=None):
    """sfm_fmatrix_ac over a list of pairs: xy_list[q] is an (n_q, 4) array of
    (x_I, y_I, x_J, y_J) pixels, wh[q] = (w_I, h_I, w_J, h_J).  Returns one
    dict per pair (F, error_max, min_nfa, n_inliers, iterations, inliers)."""
    lib = abi.load()
    off, xy, wh = _fmatrix_inputs(xy_list, wh)
    n_pairs = len(off) - 1
    res = (abi.FMatrixResult * max(n_pairs, 1))()
    inl = np.full(max(int(off[-1]), 1), -1, np.int32)
    _check(lib.sfm_fmatrix_ac(ctx.h, n_pairs, abi.ptr(off, abi.i64p), abi.ptr(xy, abi.f64p),
                              abi.ptr(wh, abi.i32p), C.byref(opts or fmatrix_opts()), res,
                              abi.ptr(inl, abi.i32p)), "sfm_fmatrix_ac")
    return _fmatrix_outputs(off, res, inl)


def sparse_filter(ctx, matches_dir, opts=None):
    lib = abi.load()
    st = abi.SparseFilterStats()
    _check(lib.sfm_sparse_filter(ctx.h, _b(matches_dir), C.byref(opts or fmatrix_opts()), C.byref(st)),
           "sfm_sparse_filter")
    return st
