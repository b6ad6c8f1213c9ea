# Round 4: wave-to-SIMD placement probe, then the ping-pong matcher with the
# group taken from HW_ID (vlib/libsfm_pp2.so): parity tests and C3 A/B.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/n_pp
mkdir -p "$OUT"
timeout -k 10 60 tools/probe/simd_probe > "$OUT/simd_probe.txt" 2>&1
head -6 "$OUT/simd_probe.txt"
SFMCORE_LIB=$GRAFT_REPO_ROOT/vlib/libsfm_pp2.so timeout -k 10 300 python -u -m pytest tests/test_match_gpu.py tests/test_match_epilogue.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/tests_pp2.log" 2>&1 || { tail -30 "$OUT/tests_pp2.log"; exit 1; }
tail -3 "$OUT/tests_pp2.log"
bash tools/gpurun/match_ab.sh base vlib/libsfm_pp2.so base vlib/libsfm_pp2.so 2>&1 | tee "$OUT/match_ab2.txt"
