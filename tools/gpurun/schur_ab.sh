# Schur kernel change check: BA parity tests on the in-tree library, then the
# C4 value and the Schur phase stamps for library variants (SFMCORE_LIB):
#   tools/gpurun/schur_ab.sh <tag> base varlib/v1.so ...
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-schur}
shift
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_headline_gpu.py tests/test_radial3.py tests/test_snavely.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c3" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
ARGS="--steps 20 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for rep in 1 2; do
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    r=$(timeout -k 10 200 python -u bench.py $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" || echo "failed")
    echo "$L: $r" | tee -a "$OUT/ab.txt"
done
done
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    r=$(timeout -k 10 200 python -u tools/schur_stamps.py 2>&1 | grep -E "schur stamps|schur ms" | tr '\n' ' ' || echo "failed")
    echo "$L: $r" | tee -a "$OUT/ab.txt"
done
