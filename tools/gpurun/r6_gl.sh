# Round 6: the dataflow tasks' LDS-DMA term pipeline (tools/ab/glds.so, built
# with SFM_DF_GLDS=1): dense / RADIAL3 / C5 GPU tests on the variant, then
# dense-S and per-camera lines, default and variant alternating, and the
# variant's dense stamps.   tools/gpurun/r6_gl.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6gl}; mkdir -p "$OUT"
V=$GRAFT_REPO_ROOT/tools/ab/glds.so
SFMCORE_LIB=$V timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_seq_gpu.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --steps 3 --warmup 1"
for v in "" "$V" "" "$V"; do
  echo "== ${v:-default}"
  SFMCORE_LIB=$v timeout -k 10 300 python -u bench.py $BASE 2>&1 >/dev/null | grep -E "dense-S|per-camera"
done
SFMCORE_LIB=$V SFM_DENSE_STAMPS=1 timeout -k 10 300 python -u bench.py $BASE --no-radial3 2>&1 >/dev/null | grep "dense stamps" | tail -1
