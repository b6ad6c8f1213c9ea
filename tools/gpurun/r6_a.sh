# Round 6: the band-path contention tests, then the C5
# fixed-write-back loop with SFM_TIMING=1 (host phases summed) and problem
# dumps of consecutive calls for the offline planner replay.
#   tools/gpurun/r6_a.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6a}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT/dump"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ba_general_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "contention" > "$OUT/contention.log" 2>&1 || { tail -30 "$OUT/contention.log"; exit 1; }
tail -6 "$OUT/contention.log"
SFM_SEQ_DUMP="$OUT/dump" SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop_fixed.json" 2> "$OUT/loop_timing_fixed.err"
python3 tools/phase_sum.py "$OUT/loop_timing_fixed.err" | head -60 > "$OUT/phase_sum_fixed.txt"
head -40 "$OUT/phase_sum_fixed.txt"
grep "build_plan" "$OUT/loop_timing_fixed.err" | head -3000 | gzip > "$OUT/build_plan_lines.txt.gz"
rm -f "$OUT/loop_timing_fixed.err"
ls -la "$OUT/dump"
