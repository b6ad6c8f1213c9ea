# Round 5: GPU tier, BCR stamps and bench lines at C4 and rank 0 of N = 8,
# rocprofv3 kernel stats of both.   tools/gpurun/r5_b.sh <tag> [test -k expr]
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r5b}
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
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p1" -o c4 -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 $ARGS > /dev/null 2>&1
f=$(find "$OUT/p1" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_c4.csv"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p8" -o f8 -- python3 "$GRAFT_REPO_ROOT/bench.py" --fake-world 8 --steps 10 $ARGS > /dev/null 2>&1
f=$(find "$OUT/p8" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_fake8.csv"
rm -rf "$OUT/p1" "$OUT/p8"
python3 "$GRAFT_REPO_ROOT/tools/kstat_brief.py" "$OUT/kernel_stats_c4.csv" "$OUT/kernel_stats_fake8.csv" | tee "$OUT/kstat_brief.txt"
# the C5 loops with SFM_TIMING phase sums, and every 100th BA problem dumped (planner replay offline)
cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT/dumps"
SFM_TIMING=1 SFM_SEQ_DUMP="$OUT/dumps" timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-match --no-snavely --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline > "$OUT/loop.json" 2> "$OUT/loop_timing.err"
grep "^\[bench\] loop" "$OUT/loop_timing.err" || true
gzip -f "$OUT"/dumps/*.bin
ls -la "$OUT/dumps"
