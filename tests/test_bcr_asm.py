"""The hand-written DPP FMAs in ba_bcr.hip (diag16) are inline asm, invisible
to the compiler's hazard recognizer: compile the file for gfx950 and check the
final schedule for DPP read-after-VALU-write hazards (tools/dpp_hazard_check.py).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_bcr_dpp_schedule_has_no_hazards(tmp_path):
    out = tmp_path / "ba_bcr.s"
    src = os.path.join(ROOT, "3dreconstruction_amd", "csrc", "ba_bcr.hip")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I/opt/rocm/include",
                    "--cuda-device-only", "-S", src, "-o", str(out)], check=True, capture_output=True)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from dpp_hazard_check import check
    text = out.read_text()
    assert text.count("v_fmac_f64_dpp") >= 240, "diag16 not fully expanded"
    assert "gpr_idx" not in text, "dynamic register indexing in the BCR kernels"
    assert check(text) == []
