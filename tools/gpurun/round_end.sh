# Round-end call: the whole -m gpu tier on the in-tree library, a dense-S /
# C4 A/B of library variants, then final_prof.sh (bench line + kernel stats
# + rank-0-of-8 lines).   tools/gpurun/round_end.sh <tag> lib...
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-final}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > "$OUT/gputests.log" 2>&1 || { tail -40 "$OUT/gputests.log"; exit 1; }
tail -1 "$OUT/gputests.log"
ARGS="--steps 20 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-radial3 --no-cpu-baseline"
for L in "$@"; do
    r=$(SFMCORE_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python -u bench.py $ARGS 2>&1 >/dev/null | grep -E "^\[bench\] BA( dense-S)?:" | cut -c1-100 | tr '\n' ' ' || echo failed)
    echo "$L: $r" | tee -a "$OUT/ab.txt"
done
bash tools/gpurun/final_prof.sh "$TAG"
