# Round 6: grown-plan GPU tests, the C5 loop tests, the BA tier, then the C5
# fixed-write-back loop with SFM_TIMING=1 (host phases summed) and the bench
# loop line.   tools/gpurun/r6_b.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6b}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
    tests/test_plan_grown_gpu.py tests/test_seq_gpu.py tests/test_ba_gpu.py tests/test_headline_gpu.py \
    > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -4 "$OUT/tests.log"
SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop_fixed.json" 2> "$OUT/loop_timing_fixed.err"
python3 tools/phase_sum.py "$OUT/loop_timing_fixed.err" | head -60 > "$OUT/phase_sum_fixed.txt"
head -45 "$OUT/phase_sum_fixed.txt"
rm -f "$OUT/loop_timing_fixed.err"
ARGS="--no-match --no-snavely --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
timeout -k 10 400 python -u bench.py --steps 5 $ARGS > "$OUT/bench_loop.json" 2> "$OUT/bench_loop.err"
python3 - "$OUT/bench_loop.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k in ("loop", "loop_fixed_writeback"):
    v = d.get(k) or {}
    print(k, {a: v.get(a) for a in ("value", "unit", "seconds", "stage_seconds", "ba_lm_iters_per_s", "lm_iterations", "images_kept")})
print("C4", d["value"])
PY
