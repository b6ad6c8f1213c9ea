# BA-side check: the BA parity tests (plus the per-level back substitution
# variant once), C4 at N=1 and rank 0 of N=8, the BCR phase stamps, and a
# kernel trace of C4 turned into the per-solve timeline (kernel time vs gaps).
#   tools/gpurun/r4_ba.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4ba}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
T="tests/test_ba_gpu.py tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_snavely.py tests/test_headline_gpu.py tests/test_seq_gpu.py"
rc=0
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests.log" 2>&1 || rc=$?
tail -1 "$OUT/tests.log"
if [ $rc -ne 0 ]; then
    tail -40 "$OUT/tests.log"
    # an assertion failure (pytest exit 1) only: the same tests with one-chunk tile groups
    [ $rc -eq 1 ] && SFM_BA_TILE_GROUP=1 timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 400 \
        --timeout-method thread > "$OUT/tests_group1.log" 2>&1; tail -3 "$OUT/tests_group1.log" 2>/dev/null
    exit 1
fi
SFM_BCR_BACK_LEVELS=1 timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "c2_banded or bcr_matches or c1_scene" > "$OUT/tests_levels.log" 2>&1 || { tail -30 "$OUT/tests_levels.log"; exit 1; }
echo "per-level back substitution: $(tail -1 $OUT/tests_levels.log)"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
timeout -k 10 300 python -u bench.py --steps 20 $ARGS > "$OUT/c4.json" 2> "$OUT/c4.err" || { tail -20 "$OUT/c4.err"; exit 1; }
grep -E "^\[bench\] BA:" "$OUT/c4.err" | head -1
timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | tee "$OUT/fake8.txt"
SFM_BCR_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 $ARGS 2>&1 >/dev/null | grep "bcr stamps" | tail -1 | tee "$OUT/bcr_stamps.txt"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o c4 -- python3 -u "$GRAFT_REPO_ROOT/bench.py" \
    --steps 3 $ARGS > /dev/null 2> "$OUT/trace.err" || { tail -30 "$OUT/trace.err"; exit 1; }
f=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
python3 "$GRAFT_REPO_ROOT/tools/iter_timeline.py" "$f" > "$OUT/timeline.txt"
rm -rf "$OUT/trace"
head -40 "$OUT/timeline.txt"
