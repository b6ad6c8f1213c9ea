"""ISA checks of the exact matcher (csrc/match.hip, match_top2_kernel), built
here with hipcc for gfx950 (CPU only; no GPU needed).

* The top-2 epilogue is compiler-visible: v_min3_i32 / v_med3_i32 are
  selected from plain C min/max and no selection instruction sits inside an
  inline asm block (the compiler's hazard recognizer cannot see those).
* Every stage barrier is preceded by the wave's own LDS-DMA drain
  (s_waitcnt vmcnt(0)).  Four waves fill a stage with global_load_lds and
  every wave reads all of it, so a wave must drain its part before the
  barrier; the round-3 build had no wait at all on the stage loop's back
  edge, which made the MUTUAL results of the unrolled build differ from the
  oracle.
Both for the shipped build and the tile-loop-unrolled variant."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "3dreconstruction_amd", "csrc", "match.hip")
HIPCC = "/opt/rocm/bin/hipcc"


def _kernels(asm):
    out = {}
    for m in re.finditer(r"^(_ZN\S*match_top2_kernelILb([01])E\S*):", asm, re.M):
        end = asm.index("s_endpgm", m.end())
        out["ratio" if m.group(2) == "1" else "nn"] = asm[m.end():end]
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("unroll", [1, 2])
def test_match_epilogue_and_stage_waits(tmp_path, unroll):
    out = tmp_path / "match.s"
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I/opt/rocm/include",
                        f"-DMATCH_TILE_UNROLL={unroll}", "--cuda-device-only", "-S", SRC, "-o", str(out)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    ks = _kernels(out.read_text())
    assert set(ks) == {"ratio", "nn"}
    for name, body in ks.items():
        # no selection instruction inside an asm block
        for blk in re.findall(r";;#ASMSTART(.*?);;#ASMEND", body, re.S):
            assert "v_min" not in blk and "v_med3" not in blk, (name, blk)
        assert body.count("v_min3_i32") >= 64, name
        if name == "ratio":
            assert body.count("v_med3_i32") >= 64
        # every barrier: the wave's LDS DMA drained just before it
        lines = [ln.strip() for ln in body.splitlines()]
        bars = [i for i, ln in enumerate(lines) if ln.startswith("s_barrier")]
        assert len(bars) >= 2, name
        for i in bars:
            window = lines[max(0, i - 12):i]
            assert any(re.match(r"s_waitcnt\s+vmcnt\(0\)", ln) for ln in window), (name, unroll, window)
