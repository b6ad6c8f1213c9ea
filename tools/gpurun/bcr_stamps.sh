# BCR level stamps (SFM_BCR_STAMPS=1): per odd block phase cycles and, per
# factor window, the pivot wave's and the slowest helper's cycles.
#   tools/gpurun/bcr_stamps.sh [lib ...]   ("base" = in-tree)
set -e
cd "$GRAFT_REPO_ROOT"
ARGS="--steps 2 --warmup 1 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for L in "${@:-base}"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    echo "$L: $(SFM_BCR_STAMPS=1 timeout -k 10 200 python -u bench.py $ARGS 2>&1 >/dev/null | grep 'bcr stamps' | tail -1)"
done
