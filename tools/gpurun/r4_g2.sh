# Round-4: Schur tile groups of 2 chunks (variant) -- C4 parity, C4 A/B, the
# Schur kernel's PMC traffic; then the new per-camera RADIAL3 bench line.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4g2}; V=${2:-vlib/libsfm_g2.so}
mkdir -p "$OUT"
export TMPDIR=/tmp
SFMCORE_LIB=$GRAFT_REPO_ROOT/$V timeout -k 10 900 python -u -m pytest tests/test_ba_gpu.py tests/test_headline_gpu.py tests/test_radial3.py -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests_variant.log" 2>&1 || { tail -40 "$OUT/tests_variant.log"; exit 1; }
tail -1 "$OUT/tests_variant.log"
bash tools/gpurun/lib_ab.sh base $V | tee "$OUT/ab.txt"
A="--steps 5 --warmup 1 --no-match --no-snavely --no-loop --no-filter --no-cpu-baseline --no-dense --no-radial3"
for L in base $V; do
  unset SFMCORE_LIB; [ "$L" != base ] && export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L
  timeout -k 10 300 python -u bench.py $A > "$OUT/pmc_$(basename $L).json" 2> "$OUT/pmc_$(basename $L).err"
  echo "$L: $(grep 'pmc passes' "$OUT/pmc_$(basename $L).err" | head -1 | cut -c1-200)"
done
unset SFMCORE_LIB
R="--steps 1 --warmup 1 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense"
timeout -k 10 400 python -u bench.py $R 2>&1 >/dev/null | grep -E "radial3" | tee "$OUT/radial3.txt"
