# Round-4: which of the dense look-ahead variants solve right (LM iterations
# per dense-S solve must be 5, as the single-stream chain's): la = side
# stream, la2 = the same with agent-scope acquire / release fences in the
# chain's kernels (buffer_inv sc1 / buffer_wbl2 sc1).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4la2}
mkdir -p "$OUT"
A="--steps 1 --warmup 1 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-radial3"
for rep in 1 2 3; do
  for L in vlib/libsfm_la.so vlib/libsfm_la2.so; do
    export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L
    echo "$L: $(timeout -k 10 300 python -u bench.py $A 2>&1 >/dev/null | grep 'dense-S' | tr '\n' ' ')" | tee -a "$OUT/dense_ab.txt"
  done
done
