# Round 5: A/B of library builds (tools/build_variant.sh outputs under
# tools/ab/) on the C4 bench line and rank 0 of N = 8, interleaved, plus the
# BA GPU tests under the variants listed in $TESTV (default: all).
#   [TESTV="a.so b.so"] tools/gpurun/r5_ab.sh <tag> <variant.so>...
set -e
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for rep in 1 2; do
  for v in in-tree "$@"; do
    L=""; [ "$v" != in-tree ] && L="$GRAFT_REPO_ROOT/$v"
    SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s|^|$v N1 |" | tee -a "$OUT/ab.txt"
    SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s|^|$v rank0-of-8 |" | tee -a "$OUT/ab.txt"
  done
done
for v in ${TESTV-$@}; do
  SFMCORE_LIB=$GRAFT_REPO_ROOT/$v timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      -m gpu tests/test_ba_gpu.py tests/test_headline_gpu.py tests/test_ba_general_gpu.py > "$OUT/tests_$(basename $v .so).log" 2>&1 \
      && echo "$v tests: $(tail -1 "$OUT/tests_$(basename $v .so).log")" | tee -a "$OUT/ab.txt" \
      || { echo "$v tests FAILED: $(tail -1 "$OUT/tests_$(basename $v .so).log")" | tee -a "$OUT/ab.txt"; exit 1; }
done
