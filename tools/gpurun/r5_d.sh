# Round 5: the dense-RCS and loop lines (dense-S, RADIAL3 per-camera, C5
# fixed write-back) and a kernel-stats profile of the dense-S section.
#   tools/gpurun/r5_d.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r5d}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --steps 5 --warmup 1"
timeout -k 10 400 python -u bench.py $BASE --no-loop > "$OUT/dense.json" 2> "$OUT/dense.err"
grep -E "dense|radial3" "$OUT/dense.err" | tail -6
timeout -k 10 400 python -u bench.py $BASE --no-dense --no-radial3 > "$OUT/loop.json" 2> "$OUT/loop.err"
grep -E "loop" "$OUT/loop.err" | tail -4
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pd" -o k -- python3 "$GRAFT_REPO_ROOT/bench.py" $BASE --no-loop --no-radial3 > /dev/null 2>&1
f=$(find "$OUT/pd" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_dense.csv"
rm -rf "$OUT/pd"
python3 "$GRAFT_REPO_ROOT/tools/kstat_brief.py" "$OUT/kernel_stats_dense.csv" | tee "$OUT/kstat_dense.txt"
