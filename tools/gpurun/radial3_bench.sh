# The dense-S and RADIAL3 bench lines with a kernel trace.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3b}
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u bench.py --no-match --no-snavely --n-pt 500000 \
    --no-loop --no-pmc --no-filter --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
grep "^\[bench\]" "$OUT/bench.err" | tail -8
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
cp "$f" "$OUT/kernel_stats.csv"
head -25 "$OUT/kernel_stats.csv" | cut -d, -f1-4 | cut -c1-150
