import importlib, time, sys, json
import numpy as np
api = importlib.import_module("3dreconstruction_amd.api")
n_img = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ctx = api.Context(0)
d = api.synth_descriptors(n_img, 4096)
off = np.arange(n_img + 1, dtype=np.int64) * 4096
plan = api.MatchPlan(ctx, d, off)
pairs = api.exhaustive_pairs(n_img)
plan.run(pairs[:100], count=False)
ctx.synchronize()
for rep in range(3):
    t = time.time()
    plan.run(pairs, count=False)
    ctx.synchronize()
    dt = time.time() - t
    ms, nl = plan.last_ms()
    print(json.dumps({"pairs": len(pairs), "wall_s": dt, "pairs_per_s": len(pairs) / dt,
                      "event_ms": ms, "launches": nl,
                      "tops": len(pairs) * 2 * 128 * 4096 * 4096 / (ms * 1e-3) / 1e12}))
