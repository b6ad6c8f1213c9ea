set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_cascade.py tests/test_match_gpu.py tests/test_mvg_io.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/casc_tests.log 2>&1 || { tail -60 gpurun_out/casc_tests.log; exit 1; }
tail -3 gpurun_out/casc_tests.log
timeout -k 10 120 ./tests/cpp/facade_test > gpurun_out/facade.log 2>&1 || { tail -30 gpurun_out/facade.log; exit 1; }
tail -4 gpurun_out/facade.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 2 --no-snavely > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || { tail -20 gpurun_out/bench_c.err; exit 1; }
grep -v "^$" gpurun_out/bench_c.err | tail -12
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c -o c -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-snavely > $R/gpurun_out/prof_c.json 2> $R/gpurun_out/prof_c.err || { tail -20 $R/gpurun_out/prof_c.err; exit 1; }
grep -i casc $R/gpurun_out/prof_c/c_kernel_stats.csv | cut -c1-200
