# Round 6: the GPU tier, the C5 loop host phases (SFM_TIMING=1) and the bench
# loop lines, then library variants (tools/ab/*.so) against the in-tree build
# on the C4 and rank-0-of-8 lines.   tools/gpurun/r6_c.sh <tag> [variant.so...]
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6c}; shift || true
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpurun/tests.sh || { cp gpurun_out/gputests.log "$OUT/"; exit 1; }
cp gpurun_out/gputests.log "$OUT/gputests.log"
SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop_fixed.json" 2> "$OUT/loop_timing_fixed.err"
python3 tools/phase_sum.py "$OUT/loop_timing_fixed.err" | head -60 > "$OUT/phase_sum_fixed.txt"
head -30 "$OUT/phase_sum_fixed.txt"
rm -f "$OUT/loop_timing_fixed.err"
ARGS="--no-match --no-snavely --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
timeout -k 10 400 python -u bench.py --steps 5 $ARGS > "$OUT/bench_loop.json" 2> "$OUT/bench_loop.err"
python3 - "$OUT/bench_loop.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k in ("loop", "loop_fixed_writeback"):
    v = d.get(k) or {}
    print(k, {a: v.get(a) for a in ("value", "seconds", "ba_lm_iterations", "ba_lm_iters_per_sec_in_loop", "kept_images")}, v.get("stage_seconds"))
print("C4", d["value"])
PY
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for rep in 1 2; do
  for v in in-tree "$@"; do
    L=""; [ "$v" != in-tree ] && L="$GRAFT_REPO_ROOT/$v"
    SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s|^|$v N1 |" | tee -a "$OUT/ab.txt"
    SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s|^|$v rank0-of-8 |" | tee -a "$OUT/ab.txt"
  done
done
