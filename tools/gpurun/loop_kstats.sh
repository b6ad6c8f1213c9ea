# Kernel stats of the C5 loop in one write-back mode (quirk | fixed).
#   tools/gpurun/loop_kstats.sh <tag> <mode>
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-lk}
MODE=${2:-quirk}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p" -o lp -- python3 "$GRAFT_REPO_ROOT/tools/loop_prof.py" 300 $MODE > "$OUT/loop_$MODE.json" 2> "$OUT/loop_$MODE.err"
f=$(find "$OUT/p" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_loop_$MODE.csv"; rm -rf "$OUT/p"
# fixed mode once more with SFM_TIMING (host phases of every call, the
# adjuster's total included) and every 100th BA problem dumped
mkdir -p "$OUT/dump"
cd "$GRAFT_REPO_ROOT"
SFM_TIMING=1 SFM_SEQ_DUMP="$OUT/dump" timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > /dev/null 2> "$OUT/timing_fixed.err"
python3 tools/phase_sum.py "$OUT/timing_fixed.err" > "$OUT/phase_sum_fixed.txt"
rm -f "$OUT/timing_fixed.err"
