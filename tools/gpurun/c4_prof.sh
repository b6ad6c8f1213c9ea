set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/c4prof
mkdir -p "$OUT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p" -o c4 -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-match --no-snavely --no-pmc \
    --no-loop --no-filter --no-dense --no-radial3 > "$OUT/prof_c4.json" 2> "$OUT/prof_c4.err"
f=$(find "$OUT/p" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats_c4.csv"; rm -rf "$OUT/p"
grep "^\[bench\] BA:" "$OUT/prof_c4.err"
