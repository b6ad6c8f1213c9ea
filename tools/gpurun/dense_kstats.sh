# Kernel stats of the dense-S bench line: tools/gpurun/dense_kstats.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-dk}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p" -o dp -- python3 "$GRAFT_REPO_ROOT/tools/dense_prof.py" > "$OUT/dense.out" 2> "$OUT/dense.err"
f=$(find "$OUT/p" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_dense.csv"; rm -rf "$OUT/p"
