# General-path parity tests, then the dense-S and RADIAL3 bench lines.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-gab}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_ba_gpu.py tests/test_radial3.py tests/test_snavely.py tests/test_headline_gpu.py > "$OUT/tests.log" 2>&1 \
    || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 400 python3 -u bench.py --no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
grep "^\[bench\]" "$OUT/bench.err" | tail -8
