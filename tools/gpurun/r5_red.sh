# Round 5: A/B of library builds on the reduce kernel: bench lines (C4, rank 0
# of N = 8) interleaved, then rocprofv3 --stats per variant, reduce rows.
#   tools/gpurun/r5_red.sh <tag> <variant.so>...
set -e
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
TESTV="" bash tools/gpurun/r5_ab.sh "$TAG" "$@"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
cd /tmp
for v in in-tree "$@"; do
  L=""; [ "$v" != in-tree ] && L="$GRAFT_REPO_ROOT/$v"
  n=$(basename "$v" .so)
  for W in 1 8; do
    FW=""; [ "$W" = 8 ] && FW="--fake-world 8"
    SFMCORE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p" -o k -- python3 "$GRAFT_REPO_ROOT/bench.py" $FW --steps 10 $ARGS > /dev/null 2>&1
    f=$(find "$OUT/p" -name "*kernel_stats.csv" | head -1)
    cp "$f" "$OUT/kstat_${n}_n$W.csv"
    echo "== $n N$W" | tee -a "$OUT/red.txt"
    grep -E "reduce|schur_kernel<0, 4, 5, 52, false>" "$f" | cut -d, -f1-4 | tee -a "$OUT/red.txt"
    rm -rf "$OUT/p"
  done
done
cd "$GRAFT_REPO_ROOT"
bash tools/gpurun/tests.sh
cp gpurun_out/gputests.log "$OUT/gputests.log"
