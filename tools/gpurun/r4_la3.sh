# Round-4: the dense look-ahead with the panel's in-place L_kk store removed
# (la3) against the side-stream variant that keeps it (la): LM iterations per
# dense-S solve must stay 5; then la3's dense parity tests.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4la3}
mkdir -p "$OUT"
A="--steps 1 --warmup 1 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-radial3"
for rep in 1 2 3; do
  for L in vlib/libsfm_la3.so base vlib/libsfm_la.so; do
    unset SFMCORE_LIB; [ "$L" != base ] && export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L
    echo "$L: $(timeout -k 10 300 python -u bench.py $A 2>&1 >/dev/null | grep 'dense-S' | tr '\n' ' ')" | tee -a "$OUT/dense_ab.txt"
  done
done
export SFMCORE_LIB=$GRAFT_REPO_ROOT/vlib/libsfm_la3.so
timeout -k 10 900 python -u -m pytest tests/test_ba_general_gpu.py tests/test_radial3.py -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests_la3.log" 2>&1 || { tail -40 "$OUT/tests_la3.log"; exit 1; }
tail -1 "$OUT/tests_la3.log"
