# RADIAL3 / C4 A/B of library variants plus C4 Schur phase stamps of each:
#   tools/gpurun/r3_stamps.sh <tag> lib...
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3s}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
bash tools/gpurun/r3_ab.sh "$@"
shift
for L in "$@"; do
    export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L
    r=$(timeout -k 10 200 python -u tools/schur_stamps.py 2>&1 | grep -E "schur stamps|schur ms" | tail -2 | tr '\n' ' ' || echo "failed")
    echo "$L: $r" | tee -a "$OUT/ab.txt"
done
