# Round 4: static issue priority for one wave of each SIMD pair in the exact
# matcher (MATCH_PRIO=1: HW_ID wave slot; =2: odd workgroups), A/B on C3.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/t_prio
mkdir -p "$OUT"
SFMCORE_LIB=$GRAFT_REPO_ROOT/vlib/libsfm_prio1.so timeout -k 10 300 python -u -m pytest tests/test_match_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests_prio1.log" 2>&1 || { tail -20 "$OUT/tests_prio1.log"; exit 1; }
tail -1 "$OUT/tests_prio1.log"
bash tools/gpurun/match_ab.sh base vlib/libsfm_prio1.so vlib/libsfm_prio2.so base vlib/libsfm_prio1.so vlib/libsfm_prio2.so 2>&1 | tee "$OUT/match_ab.txt"
