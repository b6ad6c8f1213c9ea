# Round 5: the C5 fixed-write-back loop with SFM_TIMING=1, host phases summed.
#   tools/gpurun/r5_lt.sh
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/lt5
mkdir -p "$OUT"
export TMPDIR=/tmp
SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop_fixed.json" 2> "$OUT/loop_timing_fixed.err"
python3 tools/phase_sum.py "$OUT/loop_timing_fixed.err" | head -60 > "$OUT/phase_sum_fixed.txt"
head -60 "$OUT/phase_sum_fixed.txt"
