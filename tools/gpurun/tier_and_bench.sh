# GPU tier (every -m gpu test, one process) and then a bench run with the
# given extra arguments: tools/gpurun/tier_and_bench.sh <tag> [bench args...]
set -e
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread ${TESTSEL:+-k "$TESTSEL"} \
    > "$OUT/gputests.log" 2>&1 || { tail -40 "$OUT/gputests.log"; exit 1; }
tail -2 "$OUT/gputests.log"
grep -E "fixed_writeback=" "$OUT/gputests.log" || true
fi
timeout -k 10 900 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
grep "^\[bench\]" "$OUT/bench.err" | tail -25
