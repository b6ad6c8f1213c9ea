# C5 loop (both write-back modes) plain and with SFM_TIMING=1 (host phase
# times of every BA call, summed), and the fixed-mode loop's kernel stats.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-lt}
mkdir -p "$OUT"
export TMPDIR=/tmp
for mode in quirk fixed; do
timeout -k 10 300 python -u tools/loop_prof.py 300 $mode > "$OUT/loop_$mode.json" 2> "$OUT/loop_$mode.err" || { tail -20 "$OUT/loop_$mode.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/loop_$mode.json').read().strip().splitlines()[-1]); print('$mode', d['value'], d['seconds'], d['stage_seconds'], d['ba_lm_iterations'])"
SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py 300 $mode > /dev/null 2> "$OUT/loop_timing_$mode.err" || { tail -20 "$OUT/loop_timing_$mode.err"; exit 1; }
python3 tools/phase_sum.py "$OUT/loop_timing_$mode.err" | head -30 > "$OUT/phase_sum_$mode.txt"
head -16 "$OUT/phase_sum_$mode.txt"
rm -f "$OUT/loop_timing_$mode.err"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p" -o lp -- python3 "$GRAFT_REPO_ROOT/tools/loop_prof.py" 300 fixed > /dev/null 2>&1
f=$(find "$OUT/p" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_loop_fixed.csv"; rm -rf "$OUT/p"
