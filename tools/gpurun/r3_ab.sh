# RADIAL3 (80-row Schur tiles) and C4 lines for library variants:
#   tools/gpurun/r3_ab.sh <tag> lib...
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3ab}
shift
mkdir -p "$OUT"
ARGS="--steps 10 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-cpu-baseline"
for rep in 1 2; do
for L in "$@"; do
    export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L
    r=$(timeout -k 10 300 python -u bench.py $ARGS 2>&1 >/dev/null | grep -E "^\[bench\] BA( radial3)?:" | cut -c1-110 | tr '\n' ' ' || echo "failed")
    echo "$L: $r" | tee -a "$OUT/ab.txt"
done
done
