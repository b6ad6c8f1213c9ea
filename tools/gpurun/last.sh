# Last call of the round: -m gpu tier on the in-tree library, step-kernel A/B
# (kstat_ab.sh), then the default bench line.   tools/gpurun/last.sh <tag> lib...
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-last}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/gputests.log" 2>&1 || { tail -40 "$OUT/gputests.log"; exit 1; }
tail -1 "$OUT/gputests.log"
timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
grep -E "^\[bench\] (BA|match):" "$OUT/bench.err"
bash tools/gpurun/kstat_ab.sh "$TAG" "$@"
