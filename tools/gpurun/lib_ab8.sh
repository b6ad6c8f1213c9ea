# C4 BA value and rank 0's shard of N=8 for several library builds
# (SFMCORE_LIB=...), with BCR stamps once per build:
#   tools/gpurun/lib_ab8.sh lib1 lib2 ...   ("base" = the in-tree build)
set -e
cd "$GRAFT_REPO_ROOT"
ARGS="--steps 20 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    r=$(SFM_BCR_STAMPS=1 timeout -k 10 200 python -u bench.py $ARGS 2>&1 >/dev/null | grep "bcr stamps" | tail -1 || echo "failed")
    echo "$L stamps: $r"
done
for rep in 1 2; do
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    r=$(timeout -k 10 200 python -u bench.py $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" || echo "failed")
    echo "$L: $r"
    r=$(timeout -k 10 200 python -u bench.py --fake-world 8 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" || echo "failed")
    echo "$L fake8: $r"
done
done
