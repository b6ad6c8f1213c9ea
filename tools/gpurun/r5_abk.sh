# Round 5: A/B of library builds on the BCR kernels: rocprofv3 kernel trace of
# rank 0 of N = 8 and of C4 per variant, per-level means (tools/bcr_levels.py).
#   tools/gpurun/r5_abk.sh <tag> <variant.so>...
set -e
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
cd /tmp
for rep in 1 2; do
  for v in in-tree "$@"; do
    L=""; [ "$v" != in-tree ] && L="$GRAFT_REPO_ROOT/$v"
    n=$(basename "$v" .so)
    for W in 1 8; do
      FW=""; [ "$W" = 8 ] && FW="--fake-world 8"
      SFMCORE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/p" -o k -- python3 "$GRAFT_REPO_ROOT/bench.py" $FW --steps 10 $ARGS > /dev/null 2>&1
      f=$(find "$OUT/p" -name "*kernel_trace.csv" | head -1)
      echo "== $n N$W rep$rep" | tee -a "$OUT/abk.txt"
      python3 "$GRAFT_REPO_ROOT/tools/bcr_levels.py" "$f" | tee -a "$OUT/abk.txt"
      rm -rf "$OUT/p"
    done
  done
done
