# Round-4 batch 2: BA parity tests on a library variant, BCR stamps / C4 A/B /
# rank 0 of N=8 against the in-tree build, then the C5 loop phase sums.
#   tools/gpurun/r4_next.sh <tag> <variant.so>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4n}; V=${2:-vlib/libsfm_xr.so}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
T="tests/test_ba_gpu.py tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_snavely.py tests/test_headline_gpu.py"
SFMCORE_LIB=$GRAFT_REPO_ROOT/$V timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests_variant.log" 2>&1 || { tail -40 "$OUT/tests_variant.log"; exit 1; }
tail -1 "$OUT/tests_variant.log"
bash tools/gpurun/bcr_stamps.sh base vlib/libsfm_headbcr.so vlib/libsfm_xr.so $V | tee "$OUT/stamps.txt"
bash tools/gpurun/lib_ab.sh base vlib/libsfm_headbcr.so $V | tee "$OUT/ab.txt"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
for L in base vlib/libsfm_headbcr.so $V; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    echo "$L: $(timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep '^\[bench\] BA:')" | tee -a "$OUT/fake8.txt"
done
unset SFMCORE_LIB
bash tools/gpurun/loop_timing.sh $TAG/lt
