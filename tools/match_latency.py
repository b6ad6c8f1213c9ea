"""Latency of one sfm_match_dense call (4096 x 4096, RootSIFT-like), cold and
after a large BA plan has run on the same context (diagnostic)."""
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
api = importlib.import_module("3dreconstruction_amd.api")
abi = importlib.import_module("3dreconstruction_amd._abi")
ctx = api.Context(0)
d = api.synth_descriptors(2, 4096)
a, b = d[:4096], d[4096:]


def lat(tag, n=30):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        api.match_dense(ctx, a, b)
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"{tag}: median {np.median(ts):.2f} ms, min {min(ts):.2f}, max {max(ts):.2f}", flush=True)


lat("cold")
lat("warm")
import bench  # noqa: E402
sc = bench.c4_scene(200, 50_000)
plan = api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
plan.run()
plan.close()
lat("after BA")

# the loop's pattern: a fresh BA plan between matches
ts = []
for it in range(10):
    p2 = api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
    p2.run()
    p2.close()
    t = time.perf_counter()
    api.match_dense(ctx, a, b)
    ts.append((time.perf_counter() - t) * 1e3)
print("match after each fresh BA plan:", " ".join(f"{x:.2f}" for x in ts), flush=True)
ts = []
for it in range(10):
    rc, s = api.ba_solve(ctx, sc["problem"], sc["extr"].copy(), sc["intr"].copy(), sc["X"].copy())
    t = time.perf_counter()
    api.match_dense(ctx, a, b)
    ts.append((time.perf_counter() - t) * 1e3)
print("match after each sfm_ba_solve:", " ".join(f"{x:.2f}" for x in ts), flush=True)

import torch  # noqa: E402
hb = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()
db = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
out = []
for it in range(5):
    p2 = api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
    p2.run()
    p2.close()
    torch.cuda.synchronize()
    t = time.perf_counter(); db.copy_(hb, non_blocking=True); torch.cuda.synchronize(); t1 = (time.perf_counter() - t) * 1e3
    t = time.perf_counter(); api.match_dense(ctx, a, b); t2 = (time.perf_counter() - t) * 1e3
    t = time.perf_counter(); api.match_dense(ctx, a, b); t3 = (time.perf_counter() - t) * 1e3
    out.append(f"torch copy {t1:.2f} / match1 {t2:.2f} / match2 {t3:.2f}")
print("after BA plan: " + " | ".join(out), flush=True)

out = []
for it in range(4):
    p2 = api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
    p2.run()
    p2.close()
    torch.cuda.synchronize()
    t = time.perf_counter(); torch.cuda.synchronize(); t0 = (time.perf_counter() - t) * 1e3
    time.sleep(0.05)
    t = time.perf_counter(); db.copy_(hb, non_blocking=True); torch.cuda.synchronize(); t1 = (time.perf_counter() - t) * 1e3
    t = time.perf_counter(); db.copy_(hb, non_blocking=True); torch.cuda.synchronize(); t2 = (time.perf_counter() - t) * 1e3
    out.append(f"sync {t0:.2f} / sleep 50ms / copy {t1:.2f} / copy {t2:.2f}")
print("after BA plan + sleep: " + " | ".join(out), flush=True)
import gc  # noqa: E402
gc.disable()
out = []
for it in range(4):
    p2 = api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
    p2.run()
    p2.close()
    torch.cuda.synchronize()
    t = time.perf_counter(); db.copy_(hb, non_blocking=True); torch.cuda.synchronize(); t1 = (time.perf_counter() - t) * 1e3
    out.append(f"copy {t1:.2f}")
print("gc disabled: " + " | ".join(out), flush=True)
