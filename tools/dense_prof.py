#!/usr/bin/env python3
"""bench.py's dense-S line alone (random-k visibility, general points + dense
RCS), for rocprofv3: python tools/dense_prof.py [radial3]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ctx = bench.api.Context(0)
model = bench.abi.SFM_CAM_RADIAL3 if len(sys.argv) > 1 and sys.argv[1] == "radial3" else 0
print(bench.bench_dense_s(ctx, model=model)["value"])
ctx.close()
