# Round-4 batch: BA parity tests, BCR stamps + C4 A/B (base vs the round-3
# level kernel), rank 0 of N=8, the matcher unroll-2 A/B, C5 loop problem dumps
# (SFM_SEQ_DUMP) and the geometric filter under a kernel trace.
#   tools/gpurun/r4_multi.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4m}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
T="tests/test_ba_gpu.py tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_snavely.py tests/test_headline_gpu.py tests/test_seq_gpu.py"
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
bash tools/gpurun/bcr_stamps.sh base vlib/libsfm_head.so | tee "$OUT/stamps.txt"
bash tools/gpurun/lib_ab.sh base vlib/libsfm_head.so | tee "$OUT/ab.txt"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | tee "$OUT/fake8.txt"
MA="--steps 2 --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline --n-pt 20000 --n-cam 100"
SFMCORE_LIB=$GRAFT_REPO_ROOT/vlib/libsfm_roll1.so timeout -k 10 300 python -u -m pytest tests/test_match_gpu.py tests/test_headline_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/tests_roll1.log" 2>&1 || { rc=$?; tail -30 "$OUT/tests_roll1.log"; [ $rc -eq 1 ] || exit $rc; }
tail -1 "$OUT/tests_roll1.log"
for L in base vlib/libsfm_mu2.so vlib/libsfm_roll1.so vlib/libsfm_roll2.so base vlib/libsfm_roll1.so; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    echo "$L: $(timeout -k 10 200 python -u bench.py $MA 2>&1 >/dev/null | grep '^\[bench\] match' | tr '\n' ' ')" | tee -a "$OUT/match_ab.txt"
done
unset SFMCORE_LIB
mkdir -p "$OUT/dumps"
LA="--steps 1 --warmup 1 --no-match --no-snavely --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline --n-pt 20000 --n-cam 100"
SFM_SEQ_DUMP="$OUT/dumps" timeout -k 10 300 python -u bench.py $LA 2>&1 >/dev/null | grep "^\[bench\] loop" | tee "$OUT/loop.txt"
FA="--steps 1 --warmup 1 --no-match --no-snavely --no-pmc --no-loop --no-dense --no-radial3 --no-cpu-baseline --n-pt 20000 --n-cam 100"
timeout -k 10 300 python -u bench.py $FA 2>&1 >/dev/null | grep "^\[bench\] filter" | tee "$OUT/filter.txt"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pf" -o f -- python3 "$GRAFT_REPO_ROOT/bench.py" $FA > "$OUT/filter_prof.json" 2>/dev/null
f=$(find "$OUT/pf" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_filter.csv"; rm -rf "$OUT/pf"
ls -la "$OUT/dumps"
