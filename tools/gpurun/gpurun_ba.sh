set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_snavely.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { tail -40 gpurun_out/ba_tests.log; exit 1; }
tail -2 gpurun_out/ba_tests.log
timeout -k 10 300 python bench.py --steps 5 --no-match --no-cpu-baseline > gpurun_out/ba_bench.json 2> gpurun_out/ba_bench.err || { tail -20 gpurun_out/ba_bench.err; exit 1; }
grep "BA" gpurun_out/ba_bench.err
