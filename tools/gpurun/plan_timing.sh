# GPU tests, then host/device phase times of the C4 bench plan and of one
# sfm_ba_solve from host buffers (SFM_TIMING=1), then the C5 loop profile.
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-pt}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpurun/tests.sh
SFM_TIMING=1 timeout -k 10 300 python -u bench.py --no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
grep -v "^\[timing\] sfm_match" "$OUT/bench.err" | tail -12
bash tools/gpurun/loop_prof.sh "$TAG/loop" 300
