# C4 value and per-kernel averages (rocprofv3 --kernel-trace --stats) for
# library variants:  tools/gpurun/kstat_ab.sh <tag> lib...
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-kab}
shift
mkdir -p "$OUT"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for rep in 1 2; do
for L in "$@"; do
    r=$(SFMCORE_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" || echo failed)
    echo "$L: $r" | tee -a "$OUT/ab.txt"
done
done
for L in "$@"; do
    d=$OUT/p_$(basename $L .so)
    (cd /tmp && SFMCORE_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o k -- \
        python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 $ARGS > /dev/null 2>&1)
    f=$(find "$d" -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$L" <<'PY' | tee -a "$OUT/ab.txt"
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("sfm::(anonymous namespace)::", "")
    if any(k in n for k in ("schur_kernel", "step_kernel", "image_gram", "bcr_level", "reduce_kernel", "finalize")):
        print(sys.argv[2], n[:48].ljust(48), r["Calls"].rjust(5), "%.1f us" % (float(r["AverageNs"]) / 1e3))
PY
    rm -rf "$d"
done
