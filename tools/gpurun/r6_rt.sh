# Round 6: rocprofv3 kernel trace of the RADIAL3 per-camera bench line (no dense-S); per-iteration
# breakdown by kernel (tools/dense_iter.py).   tools/gpurun/r6_dt.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6rt}; mkdir -p "$OUT"
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --no-dense --steps 2 --warmup 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u bench.py $BASE > "$OUT/bench.log" 2>&1
f=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python3 tools/dense_iter.py "$f" | tee "$OUT/dense_iter.txt"
