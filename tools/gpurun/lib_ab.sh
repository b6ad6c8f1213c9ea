# C4 BA value for several library builds (SFMCORE_LIB=...): tools/gpurun/lib_ab.sh lib1 lib2 ...
set -e
cd "$GRAFT_REPO_ROOT"
ARGS="--steps 20 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for rep in 1 2; do
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    r=$(timeout -k 10 200 python -u bench.py $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" || echo "failed")
    echo "$L: $r"
done
done
