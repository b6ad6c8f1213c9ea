# BCR change check: BA parity tests, then C4 (with and without BCR phase
# stamps) and rank 0's shard of N=8.  Outputs under gpurun_out/<tag>/.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-bcr}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_ba_gpu.py tests/test_headline_gpu.py tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_snavely.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c3" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:"
SFM_BCR_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 5 $ARGS 2>&1 >/dev/null | grep "bcr stamps"
timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:"
