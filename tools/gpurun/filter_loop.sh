# Bench line without the matcher / BAL / PMC sections (C4 + filter + CPU
# baselines), then the C5 loop profile.  Outputs under gpurun_out/<tag>/.
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-fl}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py --no-match --no-snavely --no-loop --no-pmc > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
tail -5 "$OUT/bench.err"
bash tools/gpurun/loop_prof.sh "$TAG/loop" 300
