# Bench line (default flags) + rocprofv3 --kernel-trace --stats of a short run
# of the same sections (kernel_stats.csv) and of the C4 BA alone
# (kernel_stats_c4.csv: the roofline kernel's average launch).  Outputs under gpurun_out/<tag>/.
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o ba -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-match --no-snavely --no-pmc \
    > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { tail -30 "$OUT/prof_bench.err"; exit 1; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats.csv"
# the C4 BA alone: its schur_kernel average is the roofline's per-launch time
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o c4 -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-match --no-snavely --no-pmc \
    --no-loop --no-filter --no-dense --no-radial3 > "$OUT/prof_c4.json" 2> "$OUT/prof_c4.err" || { tail -30 "$OUT/prof_c4.err"; exit 1; }
f=$(find "$OUT/prof_c4" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats_c4.csv"
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:24]:
    print(r['Name'][:70].ljust(70), r['Calls'].rjust(6), '%10.1f' % (float(r['AverageNs']) / 1e3), '%6.2f' % float(r['Percentage']))
PY
