# Round 6: dense-S under a kernel trace -- one factorisation's timeline
# (panel / narrow update / trailing update launches, kernel time vs gaps).
#   tools/gpurun/r6_dtrace.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6dt}
mkdir -p "$OUT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o dt -- python3 -u "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 \
    --no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-radial3 \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
cp "$f" "$OUT/kernel_trace.csv" && rm -rf "$OUT/prof"
python3 "$GRAFT_REPO_ROOT/tools/dense_timeline.py" "$OUT/kernel_trace.csv" | tee "$OUT/dense_timeline.txt"
gzip -f "$OUT/kernel_trace.csv"
