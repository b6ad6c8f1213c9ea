# Round 5: A/B of library builds on the dense-RCS lines (dense-S, RADIAL3
# per-camera), interleaved, two repetitions.
#   tools/gpurun/r5_abd.sh <tag> <variant.so>...
set -e
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --steps 3 --warmup 1"
for rep in 1 2; do
  for v in in-tree "$@"; do
    L=""; [ "$v" != in-tree ] && L="$GRAFT_REPO_ROOT/$v"
    SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py $BASE 2>&1 >/dev/null | grep -E "dense-S|per-camera" | sed "s|^|$v |" | tee -a "$OUT/abd.txt"
  done
done
