# Round 4: ping-pong matcher variant (MATCH_PP=1, vlib/libsfm_pp.so): match
# parity tests on the variant, then the C3 match A/B against the in-tree build.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/n_pp
mkdir -p "$OUT"
SFMCORE_LIB=$GRAFT_REPO_ROOT/vlib/libsfm_pp.so timeout -k 10 300 python -u -m pytest tests/test_match_gpu.py tests/test_match_epilogue.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/tests_pp.log" 2>&1 || { tail -30 "$OUT/tests_pp.log"; exit 1; }
tail -3 "$OUT/tests_pp.log"
bash tools/gpurun/match_ab.sh base vlib/libsfm_pp.so base vlib/libsfm_pp.so 2>&1 | tee "$OUT/match_ab.txt"
