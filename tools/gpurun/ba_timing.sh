# BA GPU parity tests, then host/device phase times of the C4 plan and of one
# sfm_ba_solve from host buffers (SFM_TIMING=1).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-bt}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_ba_gpu.py tests/test_radial3.py tests/test_snavely.py > "$OUT/tests.log" 2>&1 \
    || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
SFM_TIMING=1 timeout -k 10 300 python -u bench.py --no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline \
    --no-dense --no-radial3 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
grep -v "^\[timing\] sfm_match" "$OUT/bench.err" | tail -14
