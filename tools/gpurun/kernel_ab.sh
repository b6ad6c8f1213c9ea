# Per-kernel average times (rocprofv3 --stats, C4 BA only) and the C4 value
# for library variants: tools/gpurun/kernel_ab.sh <kernel-regex> lib...
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RX=$1; shift
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
OUT=$GRAFT_REPO_ROOT/gpurun_out/kab
mkdir -p "$OUT"
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    v=$(timeout -k 10 200 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" || echo failed)
    d=$OUT/$(basename $L)
    rm -rf "$d"
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o k -- \
        python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 $ARGS > /dev/null 2>&1)
    f=$(find "$d" -name '*kernel_stats.csv' | head -1)
    echo "$L: $v"
    python3 - "$f" "$RX" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Name"]):
        print("   ", r["Name"].replace("sfm::(anonymous namespace)::", "")[:60], r["Calls"], "%.1f us" % (float(r["AverageNs"]) / 1e3))
PY
done
