# GPU tier, then a BA-only bench line (C4 + pcie + dense-S, no PMC).
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-tb}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpurun/tests.sh
timeout -k 10 300 python -u bench.py --no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
grep "^\[bench\]" "$OUT/bench.err" | tail -8
