# dense-S / RADIAL3 bench lines and the general-path kernel averages for
# library variants: tools/gpurun/dense_ab.sh lib...
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline"
OUT=$GRAFT_REPO_ROOT/gpurun_out/dab
mkdir -p "$OUT"
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python -u bench.py $ARGS 2> "$OUT/$(basename $L).err" > /dev/null
    echo "$L: $(grep -E '^\[bench\] BA (dense-S|radial3)' "$OUT/$(basename $L).err" | sed 's/, plan.*//' | tr '\n' ' ')"
done
