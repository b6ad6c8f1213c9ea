# One call: BA + matcher GPU tests on the in-tree library, the C4 A/B of
# BA library variants and the C3 A/B of matcher variants.
#   tools/gpurun/combo_ab.sh <tag> "<ba libs>" "<match libs>"
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-combo}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_headline_gpu.py tests/test_radial3.py tests/test_snavely.py tests/test_match_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
ARGS="--steps 20 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for rep in 1 2; do
for L in $2; do
    export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L
    r=$(timeout -k 10 200 python -u bench.py $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" || echo "failed")
    echo "$L: $r" | tee -a "$OUT/ab.txt"
done
done
MARGS="--steps 2 --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline --n-pt 20000 --n-cam 100"
for rep in 1 2; do
for L in $3; do
    export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L
    r=$(timeout -k 10 200 python -u bench.py $MARGS 2>&1 >/dev/null | grep "^\[bench\] match" | tr '\n' ' ' || echo "failed")
    echo "$L: $r" | tee -a "$OUT/ab.txt"
done
done
