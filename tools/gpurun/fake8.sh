# GPU tier, then C4 at N=1, rank 0's shard of N=8 untraced (device no-op
# exchange) and under rocprofv3, and the RADIAL3 / dense-S lines.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-f8}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline"
timeout -k 10 600 python -u bench.py --steps 10 $ARGS > "$OUT/c4.json" 2> "$OUT/c4.err" || { tail -20 "$OUT/c4.err"; exit 1; }
grep -E "^\[bench\] (BA|loop)" "$OUT/c4.err"
ARGS="$ARGS --no-dense --no-radial3"
timeout -k 10 300 python -u bench.py --fake-world 8 --steps 10 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p" -o f8 -- python3 "$GRAFT_REPO_ROOT/bench.py" --fake-world 8 --steps 10 $ARGS > /dev/null 2>&1
f=$(find "$OUT/p" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_fake8.csv"; rm -rf "$OUT/p"
