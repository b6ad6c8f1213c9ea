# Matcher A/B: the bench's C3 match lines and the match kernels' rocprofv3
# averages for library variants: tools/gpurun/match_ab.sh lib...  ("base" = in-tree)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ARGS="--no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline --n-pt 20000 --n-cam 100"
OUT=$GRAFT_REPO_ROOT/gpurun_out/mab
mkdir -p "$OUT"
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    echo "$L:"
    timeout -k 10 200 python -u bench.py --steps 2 $ARGS 2>&1 >/dev/null | grep "^\[bench\] match" || echo failed
    d=$OUT/$(basename $L)
    rm -rf "$d"
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o k -- \
        python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 $ARGS > /dev/null 2>&1)
    f=$(find "$d" -name '*kernel_stats.csv' | head -1)
    python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "match_top2" in r["Name"] or "mutual" in r["Name"]:
        print("   ", r["Name"].replace("sfm::(anonymous namespace)::", "")[:60], r["Calls"], "%.1f us" % (float(r["AverageNs"]) / 1e3),
              "total %.1f ms" % (float(r["TotalDurationNs"]) / 1e6))
PY
done
