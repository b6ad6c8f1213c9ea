# Round 6: dense dataflow tests + C5 loop stamps + loop timing.   tools/gpurun/r6_f.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6f}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
    tests/test_ba_general_gpu.py tests/test_plan_grown_gpu.py tests/test_seq_gpu.py tests/test_ba_gpu.py \
    > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
bash tools/gpurun/r6_e.sh "$TAG"
SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop_t.json" 2> "$OUT/timing.err" || { tail -20 "$OUT/timing.err"; exit 1; }
cat "$OUT/loop_t.json" | head -c 600; echo
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pd" -o k -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --no-radial3 --steps 3 --warmup 1 > /dev/null 2> "$OUT/dense_bench.err"
f=$(find "$OUT/pd" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_dense.csv"; rm -rf "$OUT/pd"
grep "dense-S" "$OUT/dense_bench.err" || true
python3 - "$OUT/kernel_stats_dense.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernels total %.1f ms" % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%9.1f ms %6s %8.1f us  %s" % (float(r["TotalDurationNs"]) / 1e6, r["Calls"], float(r["AverageNs"]) / 1e3, r["Name"][:80]))
PY
