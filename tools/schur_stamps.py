#!/usr/bin/env python3
"""Phase cycles of the C4 Schur kernel (SFM_SCHUR_STAMPS=1 diagnostic build
path): one plan, two solves; libsfmcore prints the per-chunk averages."""
import os
import sys

os.environ["SFM_SCHUR_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ctx = bench.api.Context(0)
sc = bench.c4_scene()
plan = bench.api.BAPlan(ctx, sc["problem"], sc["extr"], sc["intr"], sc["X"])
for _ in range(2):
    plan.run()
ctx.synchronize()
print("schur ms/launch", plan.info().schur_ms_total / max(plan.info().schur_launches, 1))
plan.close()
ctx.close()
