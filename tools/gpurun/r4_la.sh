# Round-4: the dense launch chain's race-free look-ahead (variant): dense
# parity tests, then dense-S A/B (in-tree / variant / variant without the
# look-ahead) and the dense kernels' rocprofv3 stats.   tools/gpurun/r4_la.sh <tag> <variant.so>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4la}; V=${2:-vlib/libsfm_la.so}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
T="tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_ba_gpu.py"
SFMCORE_LIB=$GRAFT_REPO_ROOT/$V timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests_variant.log" 2>&1 || { tail -40 "$OUT/tests_variant.log"; exit 1; }
tail -1 "$OUT/tests_variant.log"
A="--steps 1 --warmup 1 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-radial3"
for rep in 1 2; do
  for L in base $V $V:nola; do
    unset SFM_DENSE_NO_LOOKAHEAD SFMCORE_LIB
    LL=${L%:nola}
    [ "$LL" != "$L" ] && export SFM_DENSE_NO_LOOKAHEAD=1
    [ "$LL" != base ] && export SFMCORE_LIB=$GRAFT_REPO_ROOT/$LL
    echo "$L: $(timeout -k 10 300 python -u bench.py $A 2>&1 >/dev/null | grep 'dense-S' | tr '\n' ' ')" | tee -a "$OUT/dense_ab.txt"
  done
done
unset SFM_DENSE_NO_LOOKAHEAD
export SFMCORE_LIB=$GRAFT_REPO_ROOT/$V
d=$OUT/k
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o k -- python3 "$GRAFT_REPO_ROOT/bench.py" $A > /dev/null 2>&1)
f=$(find "$d" -name '*kernel_stats.csv' | head -1); cp "$f" "$OUT/kernel_stats_dense_la.csv"; rm -rf "$d"
head -12 "$OUT/kernel_stats_dense_la.csv" | cut -c1-160
