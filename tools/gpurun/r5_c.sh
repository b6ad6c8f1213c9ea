# Round 5: GPU tier (optionally -k), BCR stamps, bench lines at C4 and rank 0
# of N = 8, kernel stats and a kernel trace (per-level BCR durations).
#   tools/gpurun/r5_c.sh <tag> [test -k expr]
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r5c}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpurun/tests.sh "${2:-}" || { cp gpurun_out/gputests.log "$OUT/"; exit 1; }
cp gpurun_out/gputests.log "$OUT/gputests.log"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
SFM_BCR_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 $ARGS > /dev/null 2> "$OUT/stamps_c4.err"
grep "bcr stamps" "$OUT/stamps_c4.err" | tail -1
SFM_BCR_STAMPS=1 timeout -k 10 300 python -u bench.py --fake-world 8 --steps 5 --warmup 1 $ARGS > /dev/null 2> "$OUT/stamps_f8.err"
grep "bcr stamps" "$OUT/stamps_f8.err" | tail -1
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/N1 /" | tee -a "$OUT/fake8.txt"
timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/rank0-of-8 /" | tee -a "$OUT/fake8.txt"
done
cd /tmp
for W in 1 8; do
  FW=""; [ "$W" = 8 ] && FW="--fake-world 8"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p$W" -o k -- python3 "$GRAFT_REPO_ROOT/bench.py" $FW --steps 10 $ARGS > /dev/null 2>&1
  f=$(find "$OUT/p$W" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_n$W.csv"
  f=$(find "$OUT/p$W" -name "*kernel_trace.csv" | head -1)
  python3 "$GRAFT_REPO_ROOT/tools/bcr_levels.py" "$f" | tee "$OUT/bcr_levels_n$W.txt"
  python3 "$GRAFT_REPO_ROOT/tools/iter_gaps.py" "$f" | tee "$OUT/iter_gaps_n$W.txt"
  rm -rf "$OUT/p$W"
done
python3 "$GRAFT_REPO_ROOT/tools/kstat_brief.py" "$OUT/kernel_stats_n1.csv" "$OUT/kernel_stats_n8.csv" | tee "$OUT/kstat_brief.txt"
