"""3dreconstruction_amd — MI355X-native bundle adjustment and descriptor
matching core for the RainbowXXX/3DReconstruction SfM pipeline.

The product is the C-ABI library lib/libsfmcore.so (hand-written HIP kernels
for gfx950 + RCCL) declared in include/sfmcore.h, with the reference-shaped
C++ façade in include/sfm/*.hpp.  This Python package is only the ctypes
binding used by the tests and bench.py (see api.py).
"""
from . import _abi  # noqa: F401
