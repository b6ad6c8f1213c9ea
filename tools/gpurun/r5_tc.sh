# Round 5: A/B of planner builds (chunk target) at rank 0 of N = 4 and 8.
#   tools/gpurun/r5_tc.sh <tag> <variant.so>...
set -e
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for rep in 1 2; do
  for v in in-tree "$@"; do
    L=""; [ "$v" != in-tree ] && L="$GRAFT_REPO_ROOT/$v"
    for W in 4 8; do
      SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py --fake-world $W --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s|^|$v rank0-of-$W |" | tee -a "$OUT/ab.txt"
    done
  done
done
