# Round-4 check: GPU tier, the unrolled-matcher variant's parity tests, C4 at
# N=1 and rank 0 of N=8 (untraced), and rocprofv3 kernel stats of C4 alone.
#   tools/gpurun/r4_check.sh <tag> [variant libs for the match tests...]
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4}; shift || true
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for L in "$@"; do
    SFMCORE_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py tests/test_match_gpu.py \
        -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/vt_$(basename $L).log" 2>&1 \
        || { echo "$L: FAILED"; tail -30 "$OUT/vt_$(basename $L).log"; exit 1; }
    echo "$L: $(tail -1 $OUT/vt_$(basename $L).log)"
done
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
timeout -k 10 300 python -u bench.py --steps 20 $ARGS > "$OUT/c4.json" 2> "$OUT/c4.err" || { tail -20 "$OUT/c4.err"; exit 1; }
grep -E "^\[bench\] BA" "$OUT/c4.err" | head -3
timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | tee "$OUT/fake8.txt"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o c4 -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 $ARGS > /dev/null 2> "$OUT/prof_c4.err" || { tail -30 "$OUT/prof_c4.err"; exit 1; }
f=$(find "$OUT/prof_c4" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats_c4.csv"; rm -rf "$OUT/prof_c4"
python3 - "$OUT/kernel_stats_c4.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:20]:
    print(r['Name'].replace('sfm::(anonymous namespace)::', '')[:60].ljust(60), r['Calls'].rjust(6), '%9.1f' % (float(r['AverageNs']) / 1e3), '%6.2f' % float(r['Percentage']))
PY
