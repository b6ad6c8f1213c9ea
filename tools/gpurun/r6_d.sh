# Round 6: dense-RCS A/B (dense-S and RADIAL3 per-camera lines, in-tree vs
# variants), the dense / general GPU tests, and a kernel-stats profile of the
# C5 fixed-write-back loop.   tools/gpurun/r6_d.sh <tag> [variant.so...]
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6d}; shift || true
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
    tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_plan_grown_gpu.py tests/test_seq_gpu.py \
    > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --steps 3 --warmup 1"
for rep in 1 2; do
  for v in in-tree "$@"; do
    L=""; [ "$v" != in-tree ] && L="$GRAFT_REPO_ROOT/$v"
    SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py $BASE 2>&1 >/dev/null | grep -E "dense-S|per-camera" | sed "s|^|$v |" | tee -a "$OUT/abd.txt"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pl" -o k -- python3 "$GRAFT_REPO_ROOT/tools/loop_prof.py" 300 fixed > /dev/null 2>&1
f=$(find "$OUT/pl" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_loop_fixed.csv"; rm -rf "$OUT/pl"
python3 - "$OUT/kernel_stats_loop_fixed.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("loop kernels total %.1f ms" % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("%9.1f ms %6s  %s" % (float(r["TotalDurationNs"]) / 1e6, r["Calls"], r["Name"][:90]))
PY
