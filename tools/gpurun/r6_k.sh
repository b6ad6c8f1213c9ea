# Round 6: every dense / general / RADIAL3 / sharded / C4 GPU test (the tier's
# BA part), then dense-S and RADIAL3 per-camera lines and the dense-S dataflow
# stamps.   tools/gpurun/r6_k.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6k}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
    tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_ba_gpu.py tests/test_plan_grown_gpu.py \
    tests/test_seq_gpu.py tests/test_headline_gpu.py tests/test_snavely.py \
    > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --steps 3 --warmup 1"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py $BASE 2>&1 >/dev/null | grep -E "dense-S|per-camera" | tee -a "$OUT/ab.txt"
done
SFM_DENSE_STAMPS=1 timeout -k 10 300 python -u bench.py $BASE --no-radial3 2> "$OUT/stamps.err" > /dev/null
grep "dense stamps" "$OUT/stamps.err" | tail -2
