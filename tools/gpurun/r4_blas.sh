# Round 4: rocBLAS (dsyrk / dgemm) for the dense RCS factor's trailing update
# (SFM_DENSE_BLAS, A/B): dense parity tests through the launch chain, then
# the dense-S and per-camera RADIAL3 bench lines.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/q_blas
mkdir -p "$OUT"
for m in syrk gemm; do
  SFM_DENSE_LAUNCHES=1 SFM_DENSE_BLAS=$m timeout -k 10 400 python -u -m pytest tests/test_ba_general_gpu.py tests/test_radial3.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/tests_$m.log" 2>&1 || { tail -30 "$OUT/tests_$m.log"; exit 1; }
  tail -2 "$OUT/tests_$m.log"
done
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --n-pt 20000 --n-cam 100 --steps 2"
for rep in 1 2; do
for m in none syrk gemm; do
  SFM_DENSE_BLAS=$m timeout -k 10 400 python -u bench.py $ARGS 2>&1 >/dev/null | grep "dense-S\|radial3\|per camera" | sed "s/^/$m /" | tee -a "$OUT/ab.txt"
done
done
cd /tmp && SFM_DENSE_BLAS=syrk timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p" -o d -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS --no-radial3 > /dev/null 2>&1
f=$(find "$OUT/p" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_dense_syrk.csv"; rm -rf "$OUT/p"
