# Round 4: fixed write-back loop, untimed run and SFM_TIMING phase sums.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/w_loop
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop.json" 2> "$OUT/loop.err"
cat "$OUT/loop.json" | cut -c1-400
SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop_t.json" 2> "$OUT/timing.err"
python3 tools/phase_sum.py "$OUT/timing.err" > "$OUT/phase_sum_fixed.txt"
head -40 "$OUT/phase_sum_fixed.txt"
