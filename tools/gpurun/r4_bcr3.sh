# Round-4 batch 3: the in-tree build's BA parity tests, then the BCR level
# kernel's rocprofv3 average for the in-tree build and two variants, the C4
# A/B, the filter with its kernel time, and the planner pool's scaling probe.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4b}
mkdir -p "$OUT"
export TMPDIR=/tmp
./tools/probe/pool_scaling > "$OUT/pool_scaling.txt" 2>&1; nproc >> "$OUT/pool_scaling.txt"; head -4 "$OUT/pool_scaling.txt"
T="tests/test_ba_gpu.py tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_snavely.py tests/test_headline_gpu.py tests/test_fmatrix.py"
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
ARGS="--steps 5 --warmup 1 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for L in base vlib/libsfm_jit.so vlib/libsfm_headbcr.so; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    d=$OUT/k_$(basename $L)
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o k -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > /dev/null 2>&1)
    f=$(find "$d" -name '*kernel_stats.csv' | head -1)
    python3 - "$L" "$f" <<'PY'
import csv, sys
tot = 0.0
for r in csv.DictReader(open(sys.argv[2])):
    if "bcr" in r["Name"]:
        n = r["Name"].replace("sfm::(anonymous namespace)::", "").split("(")[0]
        print("  %-8s %-40s %5s calls %7.1f us" % (sys.argv[1][-12:], n, r["Calls"], float(r["AverageNs"]) / 1e3))
PY
    rm -rf "$d"
done
unset SFMCORE_LIB
bash tools/gpurun/lib_ab.sh base vlib/libsfm_jit.so vlib/libsfm_headbcr.so | tee "$OUT/ab.txt"
FA="--steps 1 --warmup 1 --no-match --no-snavely --no-pmc --no-loop --no-dense --no-radial3 --no-cpu-baseline --n-pt 20000 --n-cam 100"
SFM_TIMING=1 timeout -k 10 300 python -u bench.py $FA > "$OUT/filter.json" 2> "$OUT/filter.err"
grep -E "filter|fmatrix" "$OUT/filter.err" | tail -4
