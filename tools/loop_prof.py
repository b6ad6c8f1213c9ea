#!/usr/bin/env python3
"""The C5 loop alone (bench.py's bench_loop, no CPU baseline): one JSON line
on stdout.  For profiling: run it under rocprofv3, or with SFM_TIMING=1 for
the host phase times of every BA call.
  python tools/loop_prof.py [n_images] [fixed]   (fixed: write-back without
  the Image::setIntrinsic quirk)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
fixed = len(sys.argv) > 2 and sys.argv[2] == "fixed"
ctx = bench.api.Context(0, flags=bench.abi.SFM_CTX_TUNE_HOST_MALLOC)
out = bench.bench_loop(ctx, n, cpu=False, fixed_writeback=fixed)
out.pop("images", None)
print(json.dumps(out))
ctx.close()
