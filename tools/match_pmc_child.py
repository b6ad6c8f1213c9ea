"""Counter-collection child for the exact matcher: C3-shaped synthetic
descriptors (4096 x 128 per frame), the first 2016 exhaustive pairs of 64
frames, RATIO mode, one launch after a warm-up.  Run under rocprofv3 --pmc by
tools/gpurun/match_pmc.sh."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from importlib import import_module

api = import_module("3dreconstruction_amd.api")

nf, nkp = 64, 4096
ctx = api.Context(0)
desc = api.synth_descriptors(nf, nkp)
off = np.arange(nf + 1, dtype=np.int64) * nkp
pairs = api.exhaustive_pairs(nf)
plan = api.MatchPlan(ctx, desc, off)
plan.run(pairs[:64], count=False)
plan.run(pairs, count=False)
ctx.synchronize()
print("pairs", len(pairs), "digest", plan.digest())
