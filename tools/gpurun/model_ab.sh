# C4 / BAL / RADIAL3 lines for several library builds (SFMCORE_LIB=...):
#   tools/gpurun/model_ab.sh lib1 lib2 ...   ("base" = the in-tree build)
set -e
cd "$GRAFT_REPO_ROOT"
ARGS="--steps 20 --no-match --no-loop --no-pmc --no-filter --no-dense --no-cpu-baseline"
for rep in 1 2; do
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python -u bench.py $ARGS 2>&1 >/dev/null | grep -E "^\[bench\] BA(:| snavely| radial3)" | sed "s|^|$L: |"
done
done
