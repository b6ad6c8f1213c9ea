"""Cascade matcher timing for A/B library variants (SFMCORE_LIB=...):
index + match over all pairs of the first N C3 frames; prints kernel ms."""
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
abi = importlib.import_module("3dreconstruction_amd._abi")
api = importlib.import_module("3dreconstruction_amd.api")
nf = int(sys.argv[1]) if len(sys.argv) > 1 else 120
d = api.synth_descriptors(nf, 4096)
off = [4096 * k for k in range(nf + 1)]
pairs = api.exhaustive_pairs(nf)
ctx = api.Context(0)
plan = api.MatchPlan(ctx, d, off)
plan.run(pairs[:64], mode=abi.SFM_MATCH_CASCADE, count=False)
ctx.synchronize()
t = time.perf_counter()
plan.cascade_index(pairs)   # hash + bucket every image (the set differs from the warm-up's)
ctx.synchronize()
t_idx = time.perf_counter() - t
best = 1e9
for _ in range(3):
    t = time.perf_counter()
    plan.run(pairs, mode=abi.SFM_MATCH_CASCADE, count=False)
    ctx.synchronize()
    best = min(best, time.perf_counter() - t)
ms, _ = plan.last_ms()
print(f"{os.environ.get('SFMCORE_LIB', 'base')}: {len(pairs)} pairs, kernel {ms:.2f} ms, "
      f"{len(pairs) / best:.0f} pairs/s, index {t_idx * 1e3:.2f} ms, digest {plan.digest()}")
plan.close()
ctx.close()
