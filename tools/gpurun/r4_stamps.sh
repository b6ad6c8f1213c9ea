# Round 4: the launch-shape agreement test, dense dataflow phase stamps on
# C5-sized dense problems, and the C4 line after moving the step split into the plan.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/r_stamps
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "split_and_reduce or grown_structure or c4_bench" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
for n in 100 200 300; do
  SFM_DENSE_STAMPS=1 timeout -k 10 200 python -u tools/dense_stamps.py $n >> "$OUT/dense_stamps.txt" 2>&1
done
grep -v amdgpu.ids "$OUT/dense_stamps.txt"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | tee "$OUT/c4.txt"
