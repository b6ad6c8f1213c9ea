# C4 BA only: the bench value over 20 steps, then rocprofv3 kernel stats of a
# 5-step run (top kernels).  Output under gpurun_out/<tag>/.
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py --steps 20 $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
grep "^\[bench\] BA" "$OUT/bench.err"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o ba -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 $ARGS > /dev/null 2> "$OUT/prof.err" || { tail -20 "$OUT/prof.err"; exit 1; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats.csv"
rm -rf "$OUT/prof"
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(r['Name'][:60].ljust(60), r['Calls'].rjust(6), '%9.1f' % (float(r['AverageNs']) / 1e3), '%6.2f' % float(r['Percentage']))
PY
