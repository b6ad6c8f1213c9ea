# rank 0 of N = 8 (--fake-world 8) under a kernel trace (per-dispatch timestamps) for the
# iteration timeline: kernel time vs gaps.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-c4t}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o c4 -- python3 -u bench.py --steps 3 --fake-world 8 \
    --no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3 \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 tools/iter_timeline.py "$f" > "$OUT/timeline.txt"
cp "$f" "$OUT/kernel_trace.csv" && rm -rf "$OUT/prof"
gzip -f "$OUT/kernel_trace.csv"
cat "$OUT/timeline.txt" | head -80
