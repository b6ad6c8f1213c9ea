# Round 6: dense launch-chain changes -- dense / RADIAL3 / C4 GPU tests, then
# the dense-S trace timeline (tools/gpurun/r6_dtrace.sh).   tools/gpurun/r6_j.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6j}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
    tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_ba_gpu.py \
    > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
bash tools/gpurun/r6_dtrace.sh "$TAG"
grep "dense-S\|per-camera" "$OUT/bench.err" || true
