"""A/B of engine-shape context flags (SFM_CTX_BA_*, include/sfmcore.h) on the
C4 bench scene, at N = 1 and at rank 0 of a fake N-rank shard, interleaved:
    python tools/ab_flags.py [--steps 20] [--fake 1,8] name=flags ...
e.g.  red1=REDUCE_WAVES(1) red2=REDUCE_WAVES(2)   (flags are evaluated against
the _abi constants; "0" is the default engine).  One line per (rep, world, name)."""
import argparse
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bench = importlib.import_module("bench")
api = importlib.import_module("3dreconstruction_amd.api")
abi = importlib.import_module("3dreconstruction_amd._abi")


def flags_of(expr):
    env = {k: getattr(abi, k) for k in dir(abi) if k.startswith("SFM_CTX_")}
    env["REDUCE_WAVES"] = lambda n: ((3 if n == 4 else 2 if n == 2 else 1) << 15)
    env["STEP_LANES"] = lambda n: ((4 if n == 8 else 3 if n == 4 else 2 if n == 2 else 1) << 12)
    return int(eval(expr, {}, env))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--fake", default="1,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    variants = [(v.split("=", 1)[0], flags_of(v.split("=", 1)[1])) for v in a.variants]
    sc = bench.c4_scene(1000, 500_000)
    for rep in range(a.reps):
        for W in [int(w) for w in a.fake.split(",")]:
            for name, fl in variants:
                if W > 1:
                    ctx = api.Context(0, rank=0, world_size=W, flags=fl | abi.SFM_CTX_DIAG_NO_EXCHANGE)
                else:
                    ctx = api.Context(0, flags=fl)
                plan = api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
                plan.run()
                ctx.synchronize()
                t0 = time.perf_counter()
                it = 0
                for _ in range(a.steps):
                    _, s = plan.run()
                    it += s.iterations
                ctx.synchronize()
                dt = time.perf_counter() - t0
                print(f"rep{rep} N{W} {name}: {it / dt:.1f} LM-iters/s", flush=True)
                plan.close()
                ctx.close()


if __name__ == "__main__":
    main()
